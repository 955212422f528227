"""Autograd Functions over the HIP C-ABI: one Function per layer of the Generator.

Activations between layers are time-major frame matrices [T*B][C] (see include/autovc_hip.h);
only the mels at the boundary keep the reference's (B, 80, T) layout.  Every forward/backward
is a call into libautovc_hip.so on the caller's current stream; nothing here computes on the
CPU or through PyTorch kernels except autograd's own gradient bookkeeping.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from ._lib import ACT_NONE, ACT_RELU, ACT_TANH, call, ptr

F32 = 4  # bytes


def _dev(t):
    return t.device


def _ctx(t):
    return _lib.context(t.device)


def _stream(t):
    return _lib.stream(t.device)


def _empty(shape, like):
    return torch.empty(shape, dtype=torch.float32, device=like.device)


def _c(t):
    return None if t is None else t.contiguous()


class GradSink:
    """In-place parameter gradients (AutoEncoder.train_step sets one for its forward + backward).

    Without a sink every backward returns fresh parameter gradients and autograd adds each into
    `p.grad` with a separate elementwise launch (~130 per training step).  With a sink, a layer's
    backward accumulates its parameter gradients straight into `p.grad` (the views of the flat
    gradient, AutoEncoder._ensure_flat) inside the same kernels (accumulate flag) and returns None
    for them.  The forward counts every use of a parameter (the encoder runs twice per loss,
    model.py:201); when the last use's backward has written, `notify(p)` fires -- the data-parallel
    bucketed all-reduce (dp.GradBuckets.param_ready) hangs off it."""

    def __init__(self, notify=None, comm=None, inplace=True):
        self.notify = notify
        self.comm = comm            # dp.GradBuckets (data parallel): the co-residency hooks
        self.inplace = inplace      # False: only the co-residency hooks (autograd accumulates gradients)
        self.uses = {}
        self.recurrences = 0        # persistent LSTM backwards still to come (their forwards ran)

    def recurrence_begin(self):
        if self.comm is not None:
            self.comm.before_recurrence()

    def recurrence_end(self):
        self.recurrences -= 1
        if self.comm is not None:
            self.comm.after_recurrence(self.recurrences)

    def use(self, *params):
        for p in params:
            if p is not None and p.requires_grad:
                self.uses[id(p)] = self.uses.get(id(p), 0) + 1

    def done(self, p):
        n = self.uses.get(id(p), 1) - 1
        self.uses[id(p)] = n
        if n <= 0 and self.notify is not None:
            self.notify(p)


_sink: GradSink | None = None


def set_grad_sink(sink: GradSink | None):
    global _sink
    _sink = sink


def _use(*params):
    if _sink is not None:
        _sink.use(*params)


def _persistent_bptt(T, B, H):
    """Will avc_lstm_backward at (T, B, H) be a persistent launch (avc_bptt_persist_eligible, a
    cached lookup in the library; asked at both ends, so a toggle in between is seen)?  Only those
    need the co-residency hooks: the other backwards are ordinary launches a collective may run
    beside."""
    return H != 32 and bool(_lib.load().avc_bptt_persist_eligible(T, B, H))


def _param_grads(params, needs):
    """Gradient buffers for a layer's parameters: their own `.grad` (in place, accumulating) when
    a sink is active and every needed one exists, else fresh tensors.  Returns (buffers, direct)."""
    if _sink is not None and _sink.inplace and all(p.grad is not None and p.grad.is_contiguous() and p.grad.shape == p.shape
                                 for p, n in zip(params, needs) if n and p is not None):
        return [p.grad if (n and p is not None) else None for p, n in zip(params, needs)], True
    return [torch.empty_like(p) if (n and p is not None) else None for p, n in zip(params, needs)], False


def _param_done(params, bufs, direct):
    """What backward returns for the parameters: None (written in place; the sink is told) or the
    fresh gradients."""
    if not direct:
        return bufs
    for p, b in zip(params, bufs):
        if b is not None:
            _sink.done(p)
    return [None] * len(bufs)


class FramesFromMel(torch.autograd.Function):
    """x (B,cm,T) [+ emb (B,ce) broadcast over T] -> frames [T*B][cm+ce]
    (encoder.py:65-66 concat; model.py:127 transpose)."""

    @staticmethod
    def forward(ctx, x, emb):
        x = x.contiguous()
        B, cm, T = x.shape
        ce = 0 if emb is None else emb.shape[1]
        emb = _c(emb)
        out = _empty((T * B, cm + ce), x)
        call("avc_frames_from_mel", T, B, cm, ptr(x), ce, ptr(emb), ptr(out), _stream(x))
        ctx.dims = (T, B, cm, ce)
        return out

    @staticmethod
    def backward(ctx, d):
        T, B, cm, ce = ctx.dims
        d = d.contiguous()
        dx = _empty((B, cm, T), d) if ctx.needs_input_grad[0] else None
        de = _empty((B, ce), d) if (ce and ctx.needs_input_grad[1]) else None
        if dx is not None or de is not None:
            call("avc_frames_from_mel_backward", T, B, cm, ce, ptr(d), cm + ce, ptr(dx), ptr(de), 0,
                 _stream(d))
        return dx, de


class MelFromFrames(torch.autograd.Function):
    """frames [T*B][cm] -> (B, cm, T)  (decoder output transpose, model.py:127)."""

    @staticmethod
    def forward(ctx, fr, T, B):
        fr = fr.contiguous()
        cm = fr.shape[1]
        out = _empty((B, cm, T), fr)
        call("avc_mel_from_frames", T, B, cm, ptr(fr), ptr(out), _stream(fr))
        ctx.dims = (T, B, cm)
        return out

    @staticmethod
    def backward(ctx, d):
        T, B, cm = ctx.dims
        d = d.contiguous()
        dfr = _empty((T * B, cm), d)
        call("avc_frames_from_mel", T, B, cm, ptr(d), 0, None, ptr(dfr), _stream(d))
        return dfr, None, None


# AUTOVC_AMAX_CHAIN=0: consumers ignore the recorded words (A/B measurements)
_AMAX_CHAIN = os.environ.get("AUTOVC_AMAX_CHAIN", "1") != "0"


def _wptr(t):
    """Device pointer of a device-word tensor (int32), None -> NULL."""
    return None if t is None else t.data_ptr()


def _amax_of(x):
    """The max words a ConvBNAct forward recorded for x (its output), if x is that very tensor
    and unmodified since (same version counter); else None (the consumer scans x itself)."""
    rec = getattr(x, "_avc_amax", None)
    if rec is None or rec[1] != x._version or not _AMAX_CHAIN:
        return None
    return rec[0]


# AUTOVC_FRAG_CHAIN=1: conv -> conv chains of the per-layer path also hand over the split image
# (off by default: it measured no C3 gain, and a handed-over image cannot hold |x| >= 65504, which
# the fp32 hand-over's guard-scaled split of the consumer handles)
_FRAG_CHAIN = os.environ.get("AUTOVC_FRAG_CHAIN", "0") == "1"
_frag_ok_cache = {}


def frag_chain_ok(T, B, cin):
    """Can a conv over [T*B][cin] frames take its input as a split image (avc_conv_frag_chain_ok)?"""
    key = (T, B, cin)
    ok = _frag_ok_cache.get(key)
    if ok is None:
        ok = _frag_ok_cache[key] = bool(_lib.load().avc_conv_frag_chain_ok(T, B, cin, 8))
    return ok and _FRAG_CHAIN


# AUTOVC_WGRAD_IMAGE=0: the per-layer path's conv forwards stop handing their weight gradients the
# split of x (avc_conv_bn_act_forward_wg / _backward_wg; bit-identical either way, round 6)
_WGRAD_IMAGE = os.environ.get("AUTOVC_WGRAD_IMAGE", "1") != "0"
_wimg_cache = {}


def wgrad_image_bytes(T, B, cin, cout):
    """Bytes of x's weight-gradient split image for this conv shape (0: not available)."""
    if not _WGRAD_IMAGE:
        return 0
    key = (T, B, cin, cout)
    n = _wimg_cache.get(key)
    if n is None:
        n = _wimg_cache[key] = int(_lib.load().avc_conv_wgrad_image_bytes(T, B, cin, cout))
    return n


def _take_frag(x):
    """The split image a ConvBNAct forward emitted for x (its output), if x is that very tensor and
    unmodified since; the record is dropped once taken (one consumer per activation)."""
    rec = x.__dict__.pop("_avc_frag", None)
    if rec is None or rec[1] != x._version or not _FRAG_CHAIN:
        return None
    return rec[0]


class ConvBNAct(torch.autograd.Function):
    """ConvNorm(k=5,p=2) -> BatchNorm1d -> act [+ residual]  (net_layers.py:39-49,
    encoder.py:69-70, decoder.py:69-70, postnet.py:54-61, model.py:131-132).

    emit_frag: the caller's next op is a conv of the same frames (a conv -> conv chain): the
    output is also written as the split-f16 image that conv's product streams, so the consumer
    skips its range scan and its split of x (avc_conv_bn_act_forward_frag; bit-identical)."""

    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, running_mean, running_var, training, momentum,
                eps, act, residual, T, B, emit_frag=False):
        x_frag = _take_frag(x)
        x = x.contiguous()
        cout, cin, _ = weight.shape
        y_pre = _empty((T * B, cout), x)
        out = _empty((T * B, cout), x)
        mean = _empty((cout,), x)
        invstd = _empty((cout,), x)
        # max words of the activation, carried from layer to layer (conv -> conv chains): the
        # producer records them while writing; the consumer skips its own scans of x
        x_amax = _amax_of(x)
        out_amax = torch.empty(4, dtype=torch.int32, device=x.device)
        if x_frag is not None and not frag_chain_ok(T, B, cin):
            x_frag = None
        out_frag = None
        if emit_frag and frag_chain_ok(T, B, cout):
            out_frag = torch.empty(int(_lib.load().avc_act_frag_bytes(T * B, cout)), dtype=torch.uint8,
                                   device=x.device)
        # the weight gradient's split of x, written by the pass that splits x for this product
        # (x's max words set its scale); the backward then skips its own split of x
        x_wimg = None
        if ctx.needs_input_grad[1] and x_amax is not None and x_frag is None:
            nb = wgrad_image_bytes(T, B, cin, cout)
            if nb:
                x_wimg = torch.empty(nb, dtype=torch.uint8, device=x.device)
        args = (_ctx(x), T, B, cin, cout, ptr(x), _wptr(x_frag), ptr(weight.contiguous()), ptr(_c(bias)),
                ptr(gamma), ptr(beta), ptr(running_mean), ptr(running_var), int(training), float(momentum),
                float(eps), act, ptr(_c(residual)), ptr(y_pre), ptr(out), _wptr(out_frag), ptr(mean), ptr(invstd),
                _wptr(x_amax), _wptr(out_amax))
        if x_wimg is not None:
            call("avc_conv_bn_act_forward_wg", *args, _wptr(x_wimg), _stream(x))
        else:
            call("avc_conv_bn_act_forward_frag", *args, _stream(x))
        ctx.x_wimg = x_wimg
        out._avc_amax = (out_amax, out._version)
        if out_frag is not None:
            out._avc_frag = (out_frag, out._version)
        _use(weight, bias, gamma, beta)
        ctx.save_for_backward(x, weight, gamma, beta, y_pre, mean, invstd)
        ctx.bias = bias
        ctx.x_amax = x_amax
        ctx.cfg = (T, B, cin, cout, int(training), act, residual is not None, bias is not None)
        return out

    @staticmethod
    def backward(ctx, d_out):
        x, weight, gamma, beta, y_pre, mean, invstd = ctx.saved_tensors
        T, B, cin, cout, training, act, has_res, has_bias = ctx.cfg
        d_out = d_out.contiguous()
        ng = ctx.needs_input_grad
        dx = _empty(x.shape, x) if ng[0] else None
        params = (weight, ctx.bias if has_bias else None, gamma, beta)
        (dw, db, dg, dbt), direct = _param_grads(params, ng[1:5])
        args = (_ctx(x), T, B, cin, cout, ptr(x), ptr(weight.contiguous()), ptr(gamma), ptr(beta), ptr(y_pre),
                ptr(mean), ptr(invstd), training, act, ptr(d_out), ptr(dx), ptr(dw), ptr(db), ptr(dg), ptr(dbt),
                2 if direct else 0, _wptr(ctx.x_amax))
        if ctx.x_wimg is not None and ng[1]:
            call("avc_conv_bn_act_backward_wg", *args, _wptr(ctx.x_wimg), _stream(x))
        else:
            call("avc_conv_bn_act_backward_ex", *args, _stream(x))
        d_res = d_out if (has_res and ng[11]) else None
        dw, db, dg, dbt = _param_done(params, (dw, db, dg, dbt), direct)
        return dx, dw, db, dg, dbt, None, None, None, None, None, None, d_res, None, None, None


def _lstm_fwd(x, w_ih, w_hh, b_ih, b_hh, y, col, ldy, reverse, save, T, B, x_amax=None, x_unit=False):
    H = w_hh.shape[1]
    din = x.shape[1]
    gates = _empty((T * B, 4 * H), x) if save else None
    cst = _empty((T * B, H), x) if save else None
    # x_amax / x_unit: what x's producer knows of its range (no scan of x; avc_lstm_forward_ex)
    call("avc_lstm_forward_ex", _ctx(x), T, B, din, H, int(reverse), ptr(x), din, ptr(w_ih.contiguous()),
         ptr(w_hh.contiguous()), ptr(b_ih), ptr(b_hh), y.data_ptr() + col * F32, ldy, ptr(gates),
         ptr(cst), _wptr(x_amax), int(x_unit), _stream(x))
    if save and _sink is not None and _persistent_bptt(T, B, H):
        _sink.recurrences += 1
    return gates, cst


def _unit_bounded(x):
    """Is x an LSTMLayer output (h = o tanh(c), every |x| <= 1), unmodified since?"""
    rec = getattr(x, "_avc_unit", None)
    return rec is not None and rec == x._version


def _lstm_bwd(x, w_ih, w_hh, b_ih, b_hh, y, col, ldy, gates, cst, d_y, d_x, reverse, acc, T, B, needs,
              x_unit=False, x_amax=None):
    H = w_hh.shape[1]
    din = x.shape[1]
    params = (w_ih, w_hh, b_ih, b_hh)
    (dwi, dwh, dbi, dbh), direct = _param_grads(params, needs)
    # the kernels write all four: fill the ones autograd does not want with scratch
    scratch = [torch.empty_like(p) if b is None else b for p, b in zip(params, (dwi, dwh, dbi, dbh))]
    # a persistent BPTT launch (decoder LSTMs at B = 128 / 256): the data-parallel all-reduce keeps
    # its collectives away from its dispatch (dp.GradBuckets, co-residency rule); other shapes are
    # ordinary launches and take no fence
    sink = _sink if _sink is not None and _persistent_bptt(T, B, H) else None
    if sink is not None:
        sink.recurrence_begin()
    call("avc_lstm_backward_ex", _ctx(x), T, B, din, H, int(reverse), ptr(x), din, ptr(w_ih.contiguous()),
         ptr(w_hh.contiguous()), y.data_ptr() + col * F32, ldy, ptr(gates), ptr(cst),
         d_y.data_ptr() + col * F32, ptr(d_x), *[ptr(t) for t in scratch], int(acc), int(direct),
         _wptr(x_amax), int(x_unit), _stream(x))
    done = tuple(_param_done(params, (dwi, dwh, dbi, dbh), direct))
    if sink is not None:
        sink.recurrence_end()
    return done


class LSTMLayer(torch.autograd.Function):
    """One unidirectional nn.LSTM layer, zero initial state (decoder.py:37,53)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, T, B, save):
        # what x's producer knows of its range (a conv's max words, or |h| <= 1 of the layer below):
        # the input projection, the input slot and the weight gradient skip their scans of x
        ctx.x_amax, ctx.x_unit = _amax_of(x), _unit_bounded(x)
        x = x.contiguous()
        H = w_hh.shape[1]
        y = _empty((T * B, H), x)
        gates, cst = _lstm_fwd(x, w_ih, w_hh, b_ih, b_hh, y, 0, H, False, save, T, B, ctx.x_amax, ctx.x_unit)
        y._avc_unit = y._version  # |y| <= 1 (_unit_bounded)
        _use(w_ih, w_hh, b_ih, b_hh)
        if save:
            ctx.save_for_backward(x, w_ih, w_hh, y, gates, cst)
            ctx.biases = (b_ih, b_hh)
        ctx.dims = (T, B)
        return y

    @staticmethod
    def backward(ctx, d_y):
        x, w_ih, w_hh, y, gates, cst = ctx.saved_tensors
        T, B = ctx.dims
        d_y = d_y.contiguous()
        d_x = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dwi, dwh, dbi, dbh = _lstm_bwd(x, w_ih, w_hh, *ctx.biases, y, 0, y.shape[1], gates, cst, d_y, d_x, False, 0,
                                       T, B, ctx.needs_input_grad[1:5], ctx.x_unit, ctx.x_amax)
        return d_x, dwi, dwh, dbi, dbh, None, None, None


class BiLSTMLayer(torch.autograd.Function):
    """One bidirectional nn.LSTM layer (encoder.py:51): output [T*B][2H] = fwd || reverse."""

    @staticmethod
    def forward(ctx, x, wi_f, wh_f, bi_f, bh_f, wi_r, wh_r, bi_r, bh_r, T, B, save):
        ctx.x_amax, ctx.x_unit = _amax_of(x), _unit_bounded(x)  # (see LSTMLayer)
        x = x.contiguous()
        H = wh_f.shape[1]
        y = _empty((T * B, 2 * H), x)
        sv = [(_empty((T * B, 4 * H), x), _empty((T * B, H), x)) if save else (None, None) for _ in range(2)]
        (g_f, c_f), (g_r, c_r) = sv
        keep = [[t.contiguous() for t in grp] for grp in ((wi_f, wh_f, bi_f, bh_f), (wi_r, wh_r, bi_r, bh_r))]
        ws = [(ctypes.c_void_p * 4)(*[ptr(t) for t in grp]) for grp in keep]
        call("avc_bilstm_forward_ex", _ctx(x), T, B, x.shape[1], H, ptr(x), x.shape[1], ws[0], ws[1], ptr(y),
             2 * H, ptr(g_f), ptr(c_f), ptr(g_r), ptr(c_r), _wptr(ctx.x_amax), int(ctx.x_unit), _stream(x))
        y._avc_unit = y._version  # |y| <= 1 (_unit_bounded)
        _use(wi_f, wh_f, bi_f, bh_f, wi_r, wh_r, bi_r, bh_r)
        if save:
            ctx.save_for_backward(x, wi_f, wh_f, wi_r, wh_r, y, g_f, c_f, g_r, c_r)
            ctx.biases = (bi_f, bh_f, bi_r, bh_r)
        ctx.dims = (T, B, H)
        return y

    @staticmethod
    def backward(ctx, d_y):
        x, wi_f, wh_f, wi_r, wh_r, y, g_f, c_f, g_r, c_r = ctx.saved_tensors
        bi_f, bh_f, bi_r, bh_r = ctx.biases
        T, B, H = ctx.dims
        d_y = d_y.contiguous()
        ng = ctx.needs_input_grad
        d_x = torch.empty_like(x) if ng[0] else None
        gf = _lstm_bwd(x, wi_f, wh_f, bi_f, bh_f, y, 0, 2 * H, g_f, c_f, d_y, d_x, False, 0, T, B, ng[1:5],
                       ctx.x_unit, ctx.x_amax)
        gr = _lstm_bwd(x, wi_r, wh_r, bi_r, bh_r, y, H, 2 * H, g_r, c_r, d_y, d_x, True, 1, T, B, ng[5:9],
                       ctx.x_unit, ctx.x_amax)
        return (d_x,) + gf + gr + (None, None, None)


class Codes(torch.autograd.Function):
    """Content codes (encoder.py:94-96, model.py:99/143): enc [T*B][64] -> (B, 32*(T//32+ceil(T/32)))."""

    @staticmethod
    def forward(ctx, enc, T, B):
        enc = enc.contiguous()
        L = 32 * (T // 32 + (T + 31) // 32)
        out = _empty((B, L), enc)
        call("avc_codes_from_encoder", T, B, ptr(enc), ptr(out), _stream(enc))
        ctx.dims = (T, B)
        return out

    @staticmethod
    def backward(ctx, d):
        T, B = ctx.dims
        d = d.contiguous()
        de = _empty((T * B, 64), d)
        call("avc_codes_from_encoder_backward", T, B, ptr(d), ptr(de), 0, _stream(d))
        return de, None, None


class DecoderInput(torch.autograd.Function):
    """Upsampled codes ++ c_trg -> [T*B][64+256]  (model.py:115-124)."""

    @staticmethod
    def forward(ctx, enc, c_trg, T, B):
        enc = enc.contiguous()
        c_trg = c_trg.contiguous()
        ce = c_trg.shape[1]
        out = _empty((T * B, 64 + ce), enc)
        call("avc_decoder_input", T, B, ptr(enc), ce, ptr(c_trg), ptr(out), _stream(enc))
        ctx.dims = (T, B, ce)
        return out

    @staticmethod
    def backward(ctx, d):
        T, B, ce = ctx.dims
        d = d.contiguous()
        de = dc = None
        if ctx.needs_input_grad[0]:
            de = _empty((T * B, 64), d)
            call("avc_decoder_input_backward", T, B, ce, ptr(d), ptr(de), 0, _stream(d))
        if ctx.needs_input_grad[1]:
            dc = _empty((B, ce), d)
            call("avc_frames_from_mel_backward", T, B, 64, ce, ptr(d), 64 + ce, None, ptr(dc), 0, _stream(d))
        return de, dc, None, None


class Linear(torch.autograd.Function):
    """LinearNorm (net_layers.py:3-20; decoder.py:77): [M][din] -> [M][dout]."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        x = x.contiguous()
        M, din = x.shape
        dout = weight.shape[0]
        y = _empty((M, dout), x)
        call("avc_linear_forward", _ctx(x), M, din, dout, ptr(x), ptr(weight.contiguous()), ptr(_c(bias)),
             ptr(y), _stream(x))
        _use(weight, bias)
        ctx.save_for_backward(x, weight)
        ctx.bias = bias
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, d_y):
        x, weight = ctx.saved_tensors
        d_y = d_y.contiguous()
        M, din = x.shape
        dout = weight.shape[0]
        ng = ctx.needs_input_grad
        dx = torch.empty_like(x) if ng[0] else None
        params = (weight, ctx.bias if ctx.has_bias else None)
        (dw, db), direct = _param_grads(params, ng[1:3])
        call("avc_linear_backward", _ctx(x), M, din, dout, ptr(x), ptr(weight.contiguous()), ptr(d_y),
             ptr(dx), ptr(dw), ptr(db), 2 if direct else 0, _stream(x))
        dw, db = _param_done(params, (dw, db), direct)
        return dx, dw, db


class Loss(torch.autograd.Function):
    """nn.MSELoss (kind 0) / nn.L1Loss (kind 1), mean reduction (model.py:286-288)."""

    @staticmethod
    def forward(ctx, a, b, kind):
        a = a.contiguous()
        b = b.contiguous()
        if a.shape != b.shape:
            raise ValueError(f"loss operands differ in shape: {tuple(a.shape)} vs {tuple(b.shape)}")
        out = _empty((), a)
        call("avc_loss_forward", _ctx(a), kind, a.numel(), ptr(a), ptr(b), ptr(out), 0, _stream(a))
        ctx.save_for_backward(a, b)
        ctx.kind = kind
        return out

    @staticmethod
    def backward(ctx, d):
        a, b = ctx.saved_tensors
        d = d.contiguous()
        ga = torch.empty_like(a) if ctx.needs_input_grad[0] else None
        gb = torch.empty_like(b) if ctx.needs_input_grad[1] else None
        call("avc_loss_backward", ctx.kind, a.numel(), ptr(a), ptr(b), ptr(d), ptr(ga), ptr(gb), 0, _stream(a))
        return ga, gb, None


def mse_loss(a, b):
    return Loss.apply(a, b, 0)


def l1_loss(a, b):
    return Loss.apply(a, b, 1)


class OverlapAverage(torch.autograd.Function):
    """(M, C, N) slices -> (C, (M-1)*step + N) NaN-padded nanmean paste (model.py:428-437); the
    backward is torch's nanmean backward (d_out / count, 0 at NaN entries)."""

    @staticmethod
    def forward(ctx, frames, step):
        frames = frames.contiguous()
        M, C, N = frames.shape
        out = _empty((C, (M - 1) * step + N), frames)
        call("avc_overlap_average", M, C, N, step, ptr(frames), ptr(out), _stream(frames))
        ctx.save_for_backward(frames)
        ctx.step = step
        return out

    @staticmethod
    def backward(ctx, d):
        (frames,) = ctx.saved_tensors
        M, C, N = frames.shape
        d = d.contiguous()
        dfr = torch.empty_like(frames)
        call("avc_overlap_average_backward", M, C, N, ctx.step, ptr(frames), ptr(d), ptr(dfr), _stream(d))
        return dfr, None


def overlap_average(frames: torch.Tensor, step: int) -> torch.Tensor:
    """(M, C, N) slices -> (C, (M-1)*step + N) NaN-padded nanmean paste (model.py:428-437)."""
    return OverlapAverage.apply(frames, step)


def gemm(a, b, bias=None, a_trans=False, b_trans=False):
    """C = op(A) op(B) (+bias) on the library's fp32 MFMA GEMM (exported for tests)."""
    a = a.contiguous()
    b = b.contiguous()
    M = a.shape[1] if a_trans else a.shape[0]
    K = a.shape[0] if a_trans else a.shape[1]
    N = b.shape[0] if b_trans else b.shape[1]
    c = _empty((M, N), a)
    call("avc_gemm", _ctx(a), M, N, K, ptr(a), int(a_trans), ptr(b), int(b_trans), ptr(_c(bias)), ptr(c), 0,
         _stream(a))
    return c


__all__ = ["FramesFromMel", "MelFromFrames", "ConvBNAct", "LSTMLayer", "BiLSTMLayer", "Codes",
           "DecoderInput", "Linear", "Loss", "mse_loss", "l1_loss", "overlap_average", "gemm",
           "ACT_NONE", "ACT_RELU", "ACT_TANH"]
