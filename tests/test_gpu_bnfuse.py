"""BatchNorm fused into the convolution's GEMM epilogue (gemm.h BnFuse, avc_bn_fuse).

Reference composition: ConvNorm -> BatchNorm1d -> relu / tanh / identity (encoder.py:69-70,
decoder.py:69-70, postnet.py:54-61), with model.py:131-132's residual on postnet's last layer.
The fused form keeps y = conv(x) in registers, forms mean / invstd in every workgroup from the
column partials behind a column-tile barrier (train mode) or from the running statistics (eval
mode), and writes the normalised output and its split image.  Every value is formed by the same
expressions in the same order as the unfused chain (GEMM -> bn_finalize -> bn_apply), so outputs,
y_pre, mean / invstd and the running statistics must be bit-identical -- at one co-resident wave of
workgroups (C2's 256) and at small grids, in both BN modes, across repeated launches (epochs) and
HIP-graph replays of the whole-Generator forward."""
import ctypes
import time

import pytest
import torch

from autovc_amd import _lib
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu

RELU, TANH, NONE = 1, 2, 0


def _fuse(on):
    _lib.call("avc_bn_fuse", int(on))


@pytest.fixture(autouse=True)
def _restore_default():
    yield
    _fuse(1)


def _conv_inputs(dev, T, B, cin, cout, residual, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(T * B, cin, generator=g)).to(dev)
    W = ((torch.rand(cout, cin, 5, generator=g) - 0.5) * 0.2).to(dev)
    bias = ((torch.rand(cout, generator=g) - 0.5) * 0.1).to(dev)
    gamma = (torch.rand(cout, generator=g) + 0.5).to(dev)
    beta = ((torch.rand(cout, generator=g) - 0.5) * 0.2).to(dev)
    rm = ((torch.rand(cout, generator=g) - 0.5) * 0.1).to(dev)
    rv = (torch.rand(cout, generator=g) + 0.5).to(dev)
    res = torch.randn(T * B, cout, generator=g).to(dev) if residual else None
    y_pre = torch.full((T * B, cout), float("nan"), device=dev)
    out = torch.full((T * B, cout), float("nan"), device=dev)
    mean = torch.zeros(cout, device=dev)
    invstd = torch.zeros(cout, device=dev)
    return x, W, bias, gamma, beta, rm, rv, res, y_pre, out, mean, invstd


def _conv_call(dev, T, B, cin, cout, act, training, t):
    x, W, bias, gamma, beta, rm, rv, res, y_pre, out, mean, invstd = t
    _lib.call("avc_conv_bn_act_forward", _lib.context(dev), T, B, cin, cout, _lib.ptr(x), _lib.ptr(W),
              _lib.ptr(bias), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(rm), _lib.ptr(rv), int(training),
              ctypes.c_float(0.1), ctypes.c_float(1e-5), act, _lib.ptr(res), _lib.ptr(y_pre), _lib.ptr(out),
              _lib.ptr(mean), _lib.ptr(invstd), _lib.stream(dev))


def _conv(dev, T, B, cin, cout, act, training, residual, seed, reps=1):
    t = _conv_inputs(dev, T, B, cin, cout, residual, seed)
    outs = []
    for _ in range(reps):
        _conv_call(dev, T, B, cin, cout, act, training, t)
        torch.cuda.synchronize()
        x, W, bias, gamma, beta, rm, rv, res, y_pre, out, mean, invstd = t
        outs.append([v.clone() for v in (out, y_pre, mean, invstd, rm, rv)])
    return outs


@pytest.mark.parametrize("T,B,cin,cout,act,residual", [
    (128, 64, 512, 512, RELU, False),   # C2 conv: 64 x 4 tiles of 128 x 128, one per CU
    (128, 64, 336, 512, RELU, False),   # encoder's first conv (cin = 80 + 256)
    (128, 64, 512, 80, NONE, True),     # postnet's last conv + residual: 64 x 64 tiles
    (128, 2, 512, 512, TANH, False),    # a small grid (8 workgroups)
    (96, 3, 80, 512, TANH, False),      # ragged rows: M = 288
])
@pytest.mark.parametrize("training", [True, False])
def test_fused_conv_bn_is_bit_identical(cuda_device, T, B, cin, cout, act, residual, training):
    _fuse(0)
    ref = _conv(cuda_device, T, B, cin, cout, act, training, residual, seed=5, reps=2)
    _fuse(1)
    got = _conv(cuda_device, T, B, cin, cout, act, training, residual, seed=5, reps=2)
    names = ["out", "y_pre", "mean", "invstd", "running_mean", "running_var"]
    bad = []
    for rep in range(2):  # the second launch runs at the next epoch of the same counters
        for n, a, b in zip(names, got[rep], ref[rep]):
            if not torch.equal(a, b):
                d = (a.double() - b.double()).abs().nan_to_num(9.0)
                bad.append((rep, n, float(d.max()), int((d > 0).sum()), a.numel()))
    assert not bad, bad
    assert torch.isfinite(got[1][0]).all()


def test_fused_conv_bn_is_taken_at_c2():
    """The C2 conv products take the fused form (one co-resident wave: 256 tiles of 128 x 128)."""
    lib = _lib.load()
    assert lib.avc_conv_frag_chain_ok(128, 64, 512, 512) == 1


def _generator(dev, training, reps, B=64, T=128):
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    ae.to(dev)
    ae.train(training)
    x = torch.from_numpy(synthetic_mel(11, B, T)).to(dev)
    c = torch.from_numpy(synthetic_embedding(12, B)).to(dev)
    outs = []
    with torch.no_grad():
        for _ in range(reps):  # eager, then captured, then replayed
            mel, post, codes = ae(x, c, c)
            torch.cuda.synchronize()
            bufs = [b.detach().clone() for n, b in ae.named_buffers() if "running" in n]
            outs.append([mel.clone(), post.clone(), codes.clone()] + bufs)
    ae.check_health()
    return outs


@pytest.mark.parametrize("training", [True, False])
def test_whole_generator_fused_bn_is_bit_identical(cuda_device, training):
    _fuse(0)
    ref = _generator(cuda_device, training, reps=4)
    _fuse(1)
    got = _generator(cuda_device, training, reps=4)
    for rep in range(4):
        for i, (a, b) in enumerate(zip(got[rep], ref[rep])):
            assert torch.equal(a, b), (rep, i, float((a.double() - b.double()).abs().max()))


def _set_handover(on):
    _lib.call("avc_split_handover", int(on))


@pytest.mark.parametrize("training", [True, False])
def test_split_handovers_are_bit_identical(cuda_device, training):
    """The encoder's last conv -> BiLSTM projection, lstm1 -> first decoder conv and lstm2 -> Linear
    hand-overs as split images written by the producers (avc_split_handover) give the bits of the
    fp32 hand-over + split pass, at C2 (B = 64: every hand-over active)."""
    try:
        _set_handover(0)
        ref = _generator(cuda_device, training, reps=3)
        _set_handover(1)
        got = _generator(cuda_device, training, reps=3)
    finally:
        _set_handover(1)
    for rep in range(3):
        for i, (a, b) in enumerate(zip(got[rep], ref[rep])):
            assert torch.equal(a, b), (rep, i, float((a.double() - b.double()).abs().max()))


def test_fused_conv_bn_beside_held_cus_completes(cuda_device):
    """The column-tile barrier beside a long kernel that holds 192 CUs on another stream (the
    co-residency hazard of DESIGN §7) with the bounded wait cut to 2^13 polls: the call never
    hangs, and its outcome is consistent -- either the grid got its CUs and the result equals the
    reference bit for bit, or the barrier gave up, the output carries NaN and the next check on
    the context raises (after which the same call gives the reference bits again).  (On the
    round-3 test box the grid completed in 0.35 ms beside the held CUs, so the give-up branch was
    not reached here.)"""
    dev = cuda_device
    ref = _conv(dev, 128, 64, 512, 512, RELU, True, False, seed=9)[0]
    t = _conv_inputs(dev, 128, 64, 512, 512, False, seed=9)  # everything ready before the CUs are held
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    _lib.call("avc_debug_persist_spin_limit", 1 << 13)
    try:
        side.wait_stream(torch.cuda.current_stream(dev))
        _lib.call("avc_debug_hog", _lib.context(dev), 192, 160 * 1024, 600_000, side.cuda_stream)
        n, t0 = ctypes.c_int(0), time.time()
        while n.value < 192 and time.time() - t0 < 20:
            _lib.call("avc_debug_hog_resident", _lib.context(dev), ctypes.byref(n))
            time.sleep(0.001)
        assert n.value == 192
        launches = _lib.persist_launches(dev)
        _conv_call(dev, 128, 64, 512, 512, RELU, True, t)  # dispatches while 192 CUs are held
        torch.cuda.synchronize()
        assert _lib.persist_launches(dev) - launches == 1  # the fused, co-resident form ran
    finally:
        _lib.call("avc_debug_persist_spin_limit", 0)
    got = [v.clone() for v in (t[9], t[8], t[10], t[11], t[5], t[6])]
    try:
        _lib.call("avc_persist_check", _lib.context(dev), _lib.stream(dev), None)
        gave_up = False
    except RuntimeError as e:
        assert "abandoned a bounded wait" in str(e)
        gave_up = True
    if gave_up:
        assert torch.isnan(got[0]).any(), "a fused conv that gave up returned only numbers"
        again = _conv(dev, 128, 64, 512, 512, RELU, True, False, seed=9)[0]
        for a, b in zip(again, ref):
            assert torch.equal(a, b)
    else:
        for a, b in zip(got, ref):
            assert torch.equal(a, b)


def test_fused_conv_bn_give_up_is_nan_and_reported(cuda_device):
    """The barrier's bounded wait, forced (avc_debug_bnf_inject): the launch gives up instead of
    waiting, its output carries NaN, the next check on the context raises, and after that reset
    the same call gives the reference bits again (a fresh counter region)."""
    dev = cuda_device
    ref = _conv(dev, 128, 64, 512, 512, RELU, True, False, seed=13)[0]
    _lib.call("avc_debug_bnf_inject", 1)
    try:
        bad = _conv(dev, 128, 64, 512, 512, RELU, True, False, seed=13)[0]
    finally:
        _lib.call("avc_debug_bnf_inject", 0)
    assert torch.isnan(bad[0]).any(), "a fused conv that gave up returned only numbers"
    with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
        _lib.call("avc_persist_check", _lib.context(dev), _lib.stream(dev), None)
    again = _conv(dev, 128, 64, 512, 512, RELU, True, False, seed=13)[0]
    for a, b in zip(again, ref):
        assert torch.equal(a, b)
