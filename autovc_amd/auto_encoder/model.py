"""Drop-in Generator: `AutoEncoder` with the reference's constructor, attributes, state_dict keys
and methods (autovc/auto_encoder/model.py:27-453), computing on hand-written gfx950 HIP kernels.

Paths:
  * inference (no autograd needed, c_trg given): ONE call into the library's whole-Generator
    forward (avc_generator_forward) — the convert() hot path;
  * everything else (training, codes-only, grad-enabled conversion): the per-layer autograd
    Functions of autovc_amd.ops, each a C-ABI forward/backward pair.
Both honour `module.training` per BatchNorm exactly like nn.BatchNorm1d (train mode uses batch
statistics and updates the running buffers; the reference never calls .eval()).
"""
from __future__ import annotations

import ctypes
import itertools
import inspect
import time

import torch
import torch.nn as nn

from .. import _lib, dp, ops
from ..hparams import AutoEncoderParams
from .decoder import Decoder
from .encoder import Encoder
from .postnet import Postnet


def _default_device():
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


_INSTANCES = itertools.count(1)
_PREP_OWNER = {}  # device -> uid of the model whose derived weights the library holds


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam semantics (amsgrad=False) on the flat parameter/gradient buffers of an
    AutoEncoder, fused with clip_grad_norm_ and the EMA of model.py:314-321 in one HIP pass
    (avc_clip_adam_ema).  state_dict() has torch Adam's layout (step/exp_avg/exp_avg_sq).

    The device counts the updates it skipped for a non-finite gradient norm, and each update's
    bias correction uses (step() calls - skips) on the device, so step() never waits for the norm.
    The host-side 'step' in ``optimizer.state[p]`` is therefore PROVISIONAL between settles: it
    counts step() calls, skipped ones included, until state_dict() or settle() folds the device
    count in.  Code that reads ``state[p]['step']`` directly should call settle() first."""

    def __init__(self, model: "AutoEncoder", lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, **_ignored):
        if amsgrad:
            raise NotImplementedError("amsgrad is not used by the reference (hparams.py:33)")
        model._ensure_flat()
        params = list(model.parameters())
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)
        self.model = model
        self.exp_avg = torch.zeros_like(model._flat_param)
        self.exp_avg_sq = torch.zeros_like(model._flat_param)
        self._step = 0  # updates requested (step() calls) since the count was last settled
        self._step_t = torch.tensor(0.0)
        # updates the device skipped for a non-finite gradient norm (adam_ema_kernel), counted on
        # the device: the kernel's bias correction uses _step - skips, so step() never waits for
        # the norm; the host count is settled when the state is read (state_dict)
        self._skips = torch.zeros(1, dtype=torch.int32, device=model._flat_param.device)
        for p, (off, n) in zip(params, model._flat_slices):
            self.state[p] = {"step": self._step_t, "exp_avg": self.exp_avg[off:off + n].view_as(p),
                             "exp_avg_sq": self.exp_avg_sq[off:off + n].view_as(p)}

    def zero_grad(self, set_to_none: bool = False):
        self.model._ensure_flat()
        self.model._flat_grad.zero_()

    @torch.no_grad()
    def step(self, closure=None, max_norm: float = 0.0, ema: torch.Tensor | None = None,
             ema_decay: float = 0.9999):
        loss = closure() if closure is not None else None
        m = self.model
        if not m._flat_valid():
            raise RuntimeError("parameters were re-allocated after the optimizer was built")
        g = self.param_groups[0]
        self._step += 1
        self._step_t.fill_(float(self._step))  # (provisional until _settle: skips not subtracted)
        norm = torch.empty((), dtype=torch.float32, device=m._flat_param.device)
        b1, b2 = g["betas"]
        # (the norm is always formed here, so the kernel's skip guard is always armed)
        _lib.call("avc_clip_adam_ema_dev", _lib.context(norm.device), m._flat_param.numel(),
                  m._flat_param.data_ptr(), m._flat_grad.data_ptr(), self.exp_avg.data_ptr(),
                  self.exp_avg_sq.data_ptr(), None if ema is None else _lib.ptr(ema), float(g["lr"]),
                  float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), self._step,
                  float(max_norm), float(ema_decay), norm.data_ptr(), self._skips.data_ptr(),
                  _lib.stream(norm.device))
        m._param_epoch += 1  # parameters changed outside torch's version counters
        self.last_grad_norm = norm
        return loss

    def _settle(self):
        """Fold the device's count of skipped updates into the host count: an update whose
        gradient norm was not finite kept parameters, moments and EMA (adam_ema_kernel), so it did
        not happen for Adam's bias correction or the checkpoint's step.  Waits for the device (only
        where the state is read)."""
        sk = int(self._skips.item())
        if sk:
            self._step -= sk
            self._skips.zero_()
        self._step_t.fill_(float(self._step))

    def settle(self):
        """Public form of _settle(): make ``state[p]['step']`` exact (waits for the device)."""
        self._settle()

    def state_dict(self):
        self._settle()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        """torch.optim.Adam's state_dict (the reference checkpoint's optimizer_state, model.py:175):
        moments copied into the flat buffers, the step count restored, param_groups settings."""
        st = state_dict["state"]
        params = list(self.model.parameters())
        if len(state_dict["param_groups"]) != 1 or len(state_dict["param_groups"][0]["params"]) != len(params):
            raise ValueError("optimizer state does not match this AutoEncoder's parameters")
        steps = set()
        for i, p in enumerate(params):
            if i in st:
                if st[i]["exp_avg"].shape != p.shape:
                    raise ValueError(f"optimizer state {i}: shape {tuple(st[i]['exp_avg'].shape)} != {tuple(p.shape)}")
                self.state[p]["exp_avg"].copy_(st[i]["exp_avg"])
                self.state[p]["exp_avg_sq"].copy_(st[i]["exp_avg_sq"])
                steps.add(int(float(st[i]["step"])))
        if len(steps) > 1:
            raise ValueError("per-parameter Adam step counts differ; the fused update keeps one")
        self._skips.zero_()
        self._step = steps.pop() if steps else 0
        self._step_t.fill_(float(self._step))
        for g, sg in zip(self.param_groups, state_dict["param_groups"]):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v


class _FusedGenerator(torch.autograd.Function):
    """Whole-Generator forward (avc_generator_forward_cached: cached derived weights, HIP-graph
    replay) as ONE autograd node, for grad-enabled calls such as convert()'s
    (voice_converter.py:172-174).  Nothing but the three inputs is saved; backward recomputes
    the per-layer forward (same kernels, same batch statistics) with the BatchNorm running
    buffers restored afterwards, so they move once per forward call as in nn.BatchNorm1d."""

    @staticmethod
    def forward(ctx, model, x, c_org, c_trg, *params):
        ctx.model = model
        ctx.params = params
        ctx.save_for_backward(x, c_org, c_trg)
        ctx.set_materialize_grads(False)
        return model._generator_forward(x, c_org, c_trg)

    @staticmethod
    def backward(ctx, d_mel, d_post, d_codes):
        model, params = ctx.model, ctx.params
        x, c_org, c_trg = ctx.saved_tensors
        need = ctx.needs_input_grad
        bufs = [b for b in model.buffers()]
        kept = [b.detach().clone() for b in bufs]
        ins = [t.detach().requires_grad_(bool(n)) for t, n in zip((x, c_org, c_trg), need[1:4])]
        with torch.enable_grad():
            outs = model._forward_layers(*ins)
        for b, k in zip(bufs, kept):  # .data: no version bump (keeps the derived-weight cache)
            b.data.copy_(k)
        pairs = [(o, d) for o, d in zip(outs, (d_mel, d_post, d_codes)) if d is not None]
        wrt = [t for t in ins if t.requires_grad] + [p for p, n in zip(params, need[4:]) if n]
        if not pairs or not wrt:
            return (None,) * (4 + len(params))
        grads = iter(torch.autograd.grad([o for o, _ in pairs], wrt, [d for _, d in pairs], allow_unused=True))
        dins = [next(grads) if t.requires_grad else None for t in ins]
        dps = [next(grads) if n else None for n in need[4:]]
        return (None, *dins, *dps)


class AutoEncoder(nn.Module):
    """Generator network (reference model.py:27): Encoder + Decoder + Postnet."""

    def __init__(self, dim_neck=AutoEncoderParams["model"]["dim_neck"],
                 dim_emb=AutoEncoderParams["model"]["dim_emb"],
                 dim_pre=AutoEncoderParams["model"]["dim_pre"],
                 freq=AutoEncoderParams["model"]["freq"], verbose=True, device=None):
        super().__init__()
        if dim_emb != 256 or dim_pre != 512:
            raise NotImplementedError("HIP Generator kernels are built for dim_emb=256, dim_pre=512")
        self.verbose = verbose
        device = _default_device() if device is None else device
        self.device = device if not isinstance(device, str) else torch.device(device)
        self.logging = {}
        self.encoder = Encoder(dim_neck, dim_emb, freq)
        self.decoder = Decoder(dim_neck, dim_emb, dim_pre)
        self.postnet = Postnet()
        self._flat_param = None
        self._flat_grad = None
        self._flat_slices = []
        self._gen_cache = None
        self._param_epoch = 0  # bumped by FusedAdam.step (it writes parameters behind torch's back)
        # grad-enabled forwards with c_trg run the fused forward under one autograd Function whose
        # backward recomputes the per-layer path; False = always the per-layer path
        self.fused_autograd = True
        self._uid = next(_INSTANCES)

    # ---- flat parameter storage (one buffer for Adam/EMA/all-reduce) -----------------------
    def _flat_valid(self):
        if self._flat_param is None:
            return False
        base = self._flat_param.data_ptr()
        for p, (off, n) in zip(self.parameters(), self._flat_slices):
            if p.data_ptr() != base + 4 * off or p.grad is None or p.grad.data_ptr() != self._flat_grad.data_ptr() + 4 * off:
                return False
        return True

    def _ensure_flat(self):
        if self._flat_valid():
            return
        params = list(self.parameters())
        dev = params[0].device
        total = sum(p.numel() for p in params)
        flat = torch.empty(total, dtype=torch.float32, device=dev)
        grad = torch.zeros(total, dtype=torch.float32, device=dev)
        slices, off = [], 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                flat[off:off + n].copy_(p.data.reshape(-1))
                p.data = flat[off:off + n].view_as(p)
                p.grad = grad[off:off + n].view_as(p)
                slices.append((off, n))
                off += n
        self._flat_param, self._flat_grad, self._flat_slices = flat, grad, slices

    def flatten_params(self):
        """model.py:379-383."""
        return torch.cat([param.data.view(-1) for param in self.parameters()], 0)

    def load_flattened_params(self, flattened_params):
        """model.py:385-392."""
        offset = 0
        for param in self.parameters():
            param.data.copy_(flattened_params[offset:offset + param.nelement()].view(param.size()))
            offset += param.nelement()
        self.weights_changed()

    def weights_changed(self):
        """Tell the fused forward that parameters were written outside torch's version counters
        (e.g. through `.data` or a raw pointer): its cached derived-weight layouts are rebuilt on
        the next call.  In-place torch ops, load_state_dict and FusedAdam need no call."""
        self._param_epoch += 1

    # ---- forward ------------------------------------------------------------------------------
    def _bns(self):
        return [m for m in self.modules() if isinstance(m, nn.BatchNorm1d)]

    def _bn_uniform(self):
        """The fused forward handles every BatchNorm in one mode with nn.BatchNorm1d defaults."""
        bns = self._bns()
        modes = {b.training for b in bns}
        return len(modes) == 1 and all(b.momentum == 0.1 and b.eps == 1e-5 and b.track_running_stats
                                       for b in bns)

    def _needs_graph(self, x, c_org, c_trg):
        return torch.is_grad_enabled() and (x.requires_grad or c_org.requires_grad or c_trg.requires_grad
                                            or any(p.requires_grad for p in self.parameters()))

    def _fast_path_ok(self, x, c_org, c_trg):
        return c_trg is not None and self._bn_uniform() and not self._needs_graph(x, c_org, c_trg)

    def _gen_params(self):
        tensors = [v for k, v in self.state_dict(keep_vars=True).items()
                   if not k.endswith("num_batches_tracked")]
        key = tuple(t.data_ptr() for t in tensors)
        dev = tensors[0].device
        if self._gen_cache is None or self._gen_cache[0] != key or _PREP_OWNER.get(dev) != self._uid:
            for t in tensors:
                _lib.ptr(t)
            # the library caches derived weight layouts per context, keyed by parameter pointers:
            # another model (whose freed storage torch may hand to this one) or moved parameters
            # must not find stale entries
            _lib.call("avc_prepared_release", _lib.context(dev))
            _PREP_OWNER[dev] = self._uid
            arr = (ctypes.c_void_p * len(tensors))(*key)
            self._gen_cache = (key, arr)
        # weights version for the library's derived-layout cache: any in-place change through
        # torch bumps a tensor's _version; FusedAdam bumps _param_epoch
        version = (self._param_epoch << 32) + sum(t._version for t in tensors)
        return self._gen_cache[1], version

    def _generator_forward(self, x, c_org, c_trg):
        B, _, T = x.shape
        training = self._bns()[0].training
        mel = torch.empty((B, 80, T), dtype=torch.float32, device=x.device)
        mel_post = torch.empty_like(mel)
        codes = torch.empty((B, 32 * (T // 32 + (T + 31) // 32)), dtype=torch.float32, device=x.device)
        params, version = self._gen_params()
        if len(params) != _lib.load().avc_generator_param_count():
            raise RuntimeError("state_dict layout does not match the library's Generator")
        _lib.call("avc_generator_forward_cached", _lib.context(x.device), T, B, params, version,
                  _lib.ptr(x), _lib.ptr(c_org), _lib.ptr(c_trg), int(training), _lib.ptr(mel),
                  _lib.ptr(mel_post), _lib.ptr(codes), _lib.stream(x.device))
        if training:  # one fused launch for the 11 counters
            torch._foreach_add_([b.num_batches_tracked for b in self._bns()], 1)
        return mel, mel_post, codes

    def check_health(self):
        """Synchronise this model's device stream and raise RuntimeError if a persistent LSTM
        recurrence launched since the last check abandoned a bounded wait (its outputs were
        written as NaN).  Every later call that reaches a persistent recurrence raises the same
        error by itself; this is the explicit form (e.g. after the last forward of a job)."""
        dev = self._flat_param.device if self._flat_param is not None else next(self.parameters()).device
        _lib.call("avc_persist_check", _lib.context(dev), _lib.stream(dev), None)

    @staticmethod
    def _check(x, c, name):
        if not x.is_cuda:
            raise RuntimeError(f"autovc_amd.AutoEncoder runs on the GPU only; {name} is on {x.device}")
        if x.dtype != torch.float32:
            raise TypeError(f"{name} must be float32, got {x.dtype}")

    def forward(self, x, c_org, c_trg):
        """model.py:68-146.  x (B,80,T) channel-first, c_org/c_trg (B,256).  Returns
        (mel_outputs, mel_outputs_postnet, content_codes), or content_codes if c_trg is None."""
        self._check(x, None, "x")
        if x.dim() != 3 or x.shape[1] != 80:
            raise ValueError(f"x must be (B, 80, T), got {tuple(x.shape)}")
        B, _, T = x.shape
        if T < self.encoder.freq:
            # the reference fails in torch.cat of an empty code list (model.py:99 / :143)
            raise ValueError("torch.cat(): expected a non-empty list of Tensors")
        c_org = c_org.to(torch.float32).contiguous()
        if c_trg is not None:
            c_trg = c_trg.to(torch.float32).contiguous()
        x = x.contiguous()
        if c_trg is not None and self._bn_uniform():
            if not self._needs_graph(x, c_org, c_trg):
                return self._generator_forward(x, c_org, c_trg)
            if self.fused_autograd:
                # grad-enabled conversion (voice_converter.py:172-174 calls self.AE(...) with grad
                # on): the same fused forward, with a recomputing backward
                return _FusedGenerator.apply(self, x, c_org, c_trg, *self.parameters())
        return self._forward_layers(x, c_org, c_trg)

    def _forward_layers(self, x, c_org, c_trg):
        """Per-layer autograd path: one Function per layer, each a C-ABI forward/backward pair."""
        B, _, T = x.shape
        save = torch.is_grad_enabled()
        enc = self.encoder.frames(x, c_org, save)
        codes = ops.Codes.apply(enc, T, B)
        if c_trg is None:
            return codes
        din = ops.DecoderInput.apply(enc, c_trg, T, B)
        melf = self.decoder.frames(din, T, B, save)
        postf = self.postnet.frames(melf, T, B, residual=melf)
        return ops.MelFromFrames.apply(melf, T, B), ops.MelFromFrames.apply(postf, T, B), codes

    # ---- checkpoints (model.py:149-181) -------------------------------------------------------
    def load(self, model_name, model_dir=AutoEncoderParams["model_dir"], device=None):
        self.device = device if device is not None else self.device
        model_path = model_dir.strip("/") + "/" + model_name
        checkpoint = torch.load(model_path, map_location=self.device, weights_only=True)
        self.load_state_dict(checkpoint["model_state"])
        self.share_memory()
        if self.verbose:
            print("Loaded auto encoder \"%s\" trained to step %d" % (model_path, checkpoint["step"]))

    def save(self, model_name, save_dir=AutoEncoderParams["learn"]["save_dir"], wandb_run=None):
        """model.py:158-181.  Data parallel: every rank must call it (the BN buffers are broadcast
        from rank 0 first); only rank 0 writes the file."""
        model_path = save_dir.strip("/") + "/" + model_name
        self._sync_bn_buffers()
        if dp.rank() != 0:
            return
        torch.save({
            "step": self.logging.get("step"),
            "model_state": {k: v.detach().clone() for k, v in self.state_dict().items()},
            "optimizer_state": self.optimiser.state_dict(),
        }, model_path)
        if wandb_run is not None:
            import wandb  # only when the caller logs to wandb
            artifact = wandb.Artifact(model_name, "AutoEncoder")
            artifact.add_file(model_path)
            wandb_run.log_artifact(artifact)

    def _sync_bn_buffers(self):
        """Data-parallel training keeps per-rank BN statistics; rank 0's are the saved ones."""
        dp.broadcast_buffers(self)

    # ---- training (model.py:184-361) ----------------------------------------------------------
    def _loss(self, X, c_org, out_decoder, out_postnet, content_codes, mu=1, lambd=1):
        """MSE(post,X) + mu*MSE(dec,X) + lambd*L1(Enc(post,c_org), codes); nothing detached."""
        reconstructed_content_codes = self(out_postnet, c_org, None)
        reconstruction_loss1 = ops.mse_loss(out_postnet, X)
        reconstruction_loss2 = ops.mse_loss(out_decoder, X)
        content_loss = ops.l1_loss(reconstructed_content_codes, content_codes)
        return reconstruction_loss1 + mu * reconstruction_loss2 + lambd * content_loss

    def configure_optimizer(self, **opt):
        params = {k: v for k, v in AutoEncoderParams["optimizer"].items()
                  if k not in ("lr_scheduler", "n_warmup_steps")}
        params.update(opt)
        self._ensure_flat()
        self.optimiser = FusedAdam(self, **params)
        self.avg_params = self._flat_param.detach().clone()
        return self.optimiser

    def train_step(self, X, c_org, ema_decay=AutoEncoderParams["learn"]["ema_decay"], max_norm=1.0):
        """One iteration of the reference loop body (model.py:304-321): forward, _loss, backward,
        [data-parallel gradient all-reduce], clip_grad_norm_(1) + Adam + EMA (one fused pass).
        Returns (loss, pre-clip total grad norm) as device scalars."""
        if getattr(self, "optimiser", None) is None or not isinstance(self.optimiser, FusedAdam):
            self.configure_optimizer()
        X = X.to(self._flat_param.device, torch.float32).contiguous()
        c_org = c_org.to(self._flat_param.device, torch.float32).contiguous()
        self._check(X, None, "X")
        # parameter gradients are accumulated in place into the flat gradient by the layers'
        # backward kernels (ops.GradSink), not returned and added by autograd
        red = self._grad_buckets() if (dp.world() > 1 or self.grad_comm is not None) else None
        sink = None
        if self.inplace_grads or red is not None:
            # without in-place gradients the sink still carries the co-residency hooks of the
            # data-parallel exchange (autograd's accumulate hooks then count the parameters)
            notify = red.param_ready if red is not None and self.inplace_grads else None
            sink = ops.GradSink(notify=notify, comm=red, inplace=self.inplace_grads)
            ops.set_grad_sink(sink)
        try:
            out_decoder, out_postnet, content_codes = self._forward_layers(X, c_org, c_org)
            loss = self._loss(X=X, c_org=c_org, out_decoder=out_decoder, out_postnet=out_postnet,
                              content_codes=content_codes)
            self.optimiser.zero_grad()
            if red is not None:
                # data parallel: bucketed RCCL all-reduce of the flat gradient, issued while
                # backward still runs but never beside a persistent launch's dispatch
                # (dp.GradBuckets, co-residency rule), then /world
                with red.armed(sink.recurrences if sink is not None else 0):
                    loss.backward()
                red.finish()
            else:
                loss.backward()
        finally:
            ops.set_grad_sink(None)
        self.optimiser.step(max_norm=max_norm, ema=self.avg_params, ema_decay=ema_decay)
        self._last_out_postnet = out_postnet.detach()  # for _log's conversion figure
        return loss.detach(), self.optimiser.last_grad_norm

    def _grad_buckets(self):
        red = getattr(self, "_reducer", None)
        if red is None or red.flat is not self._flat_grad or red.comm_key != self.grad_comm:
            if red is not None:
                red.remove()
            kw = dict(self.grad_comm or {})
            red = self._reducer = dp.GradBuckets(self.parameters(), self._flat_grad, self.bucket_bytes, **kw)
            red.comm_key = self.grad_comm
        return red

    bucket_bytes = 16 << 20  # data-parallel all-reduce bucket (≈7 buckets over the 113.7 MB gradient)
    inplace_grads = True     # train_step: layers accumulate parameter gradients in place (ops.GradSink)
    # keyword arguments of dp.GradBuckets (all_reduce, world_size, co_residency) for tests that drive
    # the bucketed exchange with a stand-in collective; None = torch.distributed when world > 1
    grad_comm = None
    _last_out_postnet = None  # train_step's postnet output, for _log's conversion figure

    def learn(self, trainloader, n_epochs=AutoEncoderParams["learn"]["n_epochs"],
              log_freq=AutoEncoderParams["learn"]["log_freq"],
              save_freq=AutoEncoderParams["learn"]["save_freq"],
              save_dir=AutoEncoderParams["learn"]["save_dir"],
              model_name=AutoEncoderParams["learn"]["model_name"],
              ema_decay=AutoEncoderParams["learn"]["ema_decay"], wandb_run=None, voice_converter=None,
              source_examples=None, target_examples=None, **opt_params):
        """Training loop of model.py:218-361 (same arguments, logging keys, save cadence and
        per-epoch ExponentialLR(0.95)); the optimizer is FusedAdam with the reference's Adam
        settings (hparams optimizer dict; like the reference, **opt_params are not applied)."""
        self.logging.update(step=0, running_loss=0.0, log_steps=0, total_time=0.0)
        # data parallel (torchrun, one process per GPU): each rank trains on its own shard of the
        # caller's loader; train_step all-reduces the gradient (dp.py)
        trainloader = dp.shard_loader(trainloader)
        N_iterations = n_epochs * len(trainloader)
        self.train()
        if wandb_run is not None:
            wandb_run.watch(self, log_freq=log_freq)
        self.criterion1 = ops.mse_loss
        self.criterion2 = ops.l1_loss
        self.configure_optimizer()
        self.lr_scheduler = torch.optim.lr_scheduler.ExponentialLR(self.optimiser, gamma=0.95)
        if self.verbose and dp.rank() == 0:
            print(f"Training Auto Encoder on {torch.cuda.get_device_name()} (cuda), {dp.world()} rank(s)...")
        for epoch in range(n_epochs):
            self.logging["step_start_time"] = time.time()
            self.logging["batch"] = 0
            dp.set_epoch(trainloader, epoch)
            for X, c_org in trainloader:
                loss, _ = self.train_step(X, c_org, ema_decay=ema_decay)
                self.logging["step"] += 1
                self.logging["running_loss"] += loss
                self.logging["log_steps"] += 1
                self.logging["epoch"] = epoch + 1
                self.logging["batch"] += 1
                self.logging["lr"] = self.optimiser.param_groups[0]["lr"]
                if self.verbose and dp.rank() == 0:
                    self.logging["total_time"] += (time.time() - self.logging["step_start_time"])
                    print(f"\rstep {self.logging['step']}/{N_iterations} | loss {float(loss):.5f}", end="")
                if (self.logging["step"] % log_freq == 0 or self.logging["step"] == N_iterations) \
                        and wandb_run is not None:
                    self._log(wandb_run, X, self._last_out_postnet)
            if self.logging["epoch"] % save_freq == 0 or self.logging["epoch"] == n_epochs:
                self.save(model_name, save_dir, wandb_run)
            if voice_converter is not None and dp.rank() == 0:
                assert source_examples is not None and target_examples is not None
                voice_converter.convert_multiple(
                    sources=source_examples, targets=target_examples,
                    save_dir="training_examples" if wandb_run is None or wandb_run.mode == "disabled" else "wandb",
                    audio_log_dict={"epoch": self.logging["epoch"], "batch": self.logging["batch"],
                                    "step": self.logging["step"]}, cut=True)
            self.lr_scheduler.step()
        if self.verbose:
            print("\n")

    def _log(self, wandb_run, X, out_postnet):
        """model.py:363-376: the running loss, then the conversion figure of the batch's first
        utterance (input vs postnet output of the step just taken)."""
        wandb_run.log({"loss": float(self.logging["running_loss"]) / self.logging["log_steps"],
                       "epoch": self.logging["epoch"], "batch": self.logging["batch"],
                       "step": self.logging["step"], "learning rate": self.logging["lr"]})
        if out_postnet is not None:
            import matplotlib.pyplot as plt  # only when logging to wandb, like the reference's use
            wandb_run.log({"Conversion": self.plot_conversion(X[0], out_postnet[0])})
            plt.close()
        self.logging["running_loss"] = 0.0
        self.logging["log_steps"] = 0

    # ---- long-form conversion (model.py:395-437) ---------------------------------------------
    def batch_forward(self, batch, c_org, c_trg, overlap=0.5):
        c_org = c_org.expand(batch.size(0), -1)
        c_trg = c_trg.expand(batch.size(0), -1)
        _, output, _ = self(batch, c_org, c_trg)
        N = batch.size(-1)
        # differentiable like the reference's pad + stack + nanmean (the graph is kept)
        return ops.overlap_average(output, int(N * (1 - overlap)))

    def plot_conversion(self, original, converted):
        import matplotlib.pyplot as plt
        fig, ax = plt.subplots(ncols=2, figsize=(20, 10))
        ax[0].matshow(original.detach().cpu().numpy())
        ax[0].set_title("Original")
        ax[1].matshow(converted.detach().cpu().numpy())
        ax[1].set_title("Reconstructed")
        return fig


AutoEncoder.learn.__allowed_args__ = inspect.getfullargspec(AutoEncoder.learn).args
AutoEncoder.learn.__allowed_kw__ = inspect.getfullargspec(torch.optim.Adam).args
