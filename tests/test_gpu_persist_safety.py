"""Safety net of the persistent weight-stationary recurrences (lstm_persist.hip).

Every wait inside a persistent launch assumes that its producer workgroups are resident.  If one is
not (another process or stream holding CUs), the wait is bounded: the launch gives up, writes the
rows it did not compute as NaN and reports itself through a pinned host word, and the next call on
the context fails with RuntimeError (AVC_ERR_DEVICE) after resetting the counter state.  The test
hook avc_debug_persist_inject makes the next launch give up at its first unsatisfied wait."""
import ctypes

import pytest
import torch

from autovc_amd import _lib
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import onehot_embedding, synthetic_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu


def _model(dev):
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    return ae.to(dev).train()


def _giveups():
    n = ctypes.c_long(0)
    _lib.call("avc_lstm_persist_status", ctypes.byref(n))
    return n.value


def _batch(dev, B=64, T=128):
    x = torch.from_numpy(synthetic_mel(71, B, T)).to(dev)
    co = torch.from_numpy(synthetic_embedding(72, B)).to(dev)
    ct = torch.from_numpy(synthetic_embedding(73, B)).to(dev)
    return x, co, ct


def test_timed_out_forward_is_nan_and_next_call_raises(cuda_device):
    ae = _model(cuda_device)
    x, co, ct = _batch(cuda_device)
    with torch.no_grad():
        ref = [o.clone() for o in ae(x, co, ct)]
        torch.cuda.synchronize()
        before = _giveups()
        _lib.call("avc_debug_persist_inject", 1)
        bad = [o.clone() for o in ae(x, co, ct)]
        torch.cuda.synchronize()
        assert _giveups() > before, "the injected launch did not give up"
        assert torch.isnan(bad[0]).any() and torch.isnan(bad[1]).any(), "timed-out launch returned numbers"
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            ae(x, co, ct)
        # state was reset: the persistent path runs again and gives the eager answer bit for bit
        # (train-mode BN normalises with batch statistics, so the NaN running buffers the failed
        # call left do not enter the outputs)
        outs = [[o.clone() for o in ae(x, co, ct)] for _ in range(3)]  # eager, capture, replay
        torch.cuda.synchronize()
    for run in outs:
        for a, b in zip(run, ref):
            assert torch.equal(a, b)
    ae.check_health()  # nothing pending


def test_check_health_reports_a_timeout(cuda_device):
    ae = _model(cuda_device)
    x, co, ct = _batch(cuda_device, 16, 64)
    with torch.no_grad():
        ae(x, co, ct)
        ae.check_health()
        _lib.call("avc_debug_persist_inject", 1)
        ae(x, co, ct)
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            ae.check_health()
        ae.check_health()  # reported once


def test_train_step_after_timeout_raises(cuda_device):
    ae = _model(cuda_device)
    B, T = 32, 64
    X = torch.from_numpy(synthetic_mel(74, B, T)).to(cuda_device)
    c = torch.from_numpy(onehot_embedding(B)).to(cuda_device)
    ae.configure_optimizer()
    ae.train_step(X, c)
    keep = [t.detach().clone() for t in (ae._flat_param, ae.optimiser.exp_avg, ae.optimiser.exp_avg_sq,
                                          ae.avg_params)]
    _lib.call("avc_debug_persist_inject", 1)
    # The give-up reaches the host word asynchronously: a later persistent call of the SAME step
    # may already see it and raise (the step stops before its update), or the step completes with
    # a non-finite loss and norm and the fused clip/Adam/EMA skips the update; the next call raises.
    # Either way nothing was updated or poisoned with NaN.
    try:
        loss, norm = ae.train_step(X, c)
    except RuntimeError as e:
        assert "abandoned a bounded wait" in str(e)
    else:
        assert not torch.isfinite(loss).item()
        assert not torch.isfinite(norm).item()
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            ae.train_step(X, c)
    for a, b in zip(keep, (ae._flat_param, ae.optimiser.exp_avg, ae.optimiser.exp_avg_sq, ae.avg_params)):
        assert torch.equal(a, b)


def test_non_finite_gradient_skips_the_update(cuda_device):
    """What a give-up leaves behind, made deterministic: a NaN in the flat gradient makes the
    fused clip/Adam/EMA skip the whole update (parameters, both moments and the EMA unchanged) and
    report a non-finite norm; a finite gradient afterwards updates normally."""
    ae = _model(cuda_device)
    B, T = 32, 64
    X = torch.from_numpy(synthetic_mel(75, B, T)).to(cuda_device)
    c = torch.from_numpy(onehot_embedding(B)).to(cuda_device)
    ae.configure_optimizer()
    ae.train_step(X, c)
    bufs = lambda: (ae._flat_param, ae.optimiser.exp_avg, ae.optimiser.exp_avg_sq, ae.avg_params)  # noqa: E731
    keep = [t.detach().clone() for t in bufs()]
    g = torch.randn_like(ae._flat_grad) * 1e-3
    ae._flat_grad.copy_(g)
    ae._flat_grad[12345] = float("nan")
    ae.optimiser.step(max_norm=1.0, ema=ae.avg_params)
    torch.cuda.synchronize()
    assert not torch.isfinite(ae.optimiser.last_grad_norm).item()
    for a, b in zip(keep, bufs()):
        assert torch.equal(a, b)
    ae._flat_grad.copy_(g)
    ae.optimiser.step(max_norm=1.0, ema=ae.avg_params)
    torch.cuda.synchronize()
    assert torch.isfinite(ae.optimiser.last_grad_norm).item()
    assert not torch.equal(keep[0], ae._flat_param)


def test_skipped_update_does_not_count_as_a_step(cuda_device):
    """A NaN-gradient step followed by a finite one gives exactly the parameters, moments, EMA and
    step count of the finite step alone (Adam's bias correction sees the updates actually applied;
    ADVICE r03)."""
    runs = []
    for with_nan in (False, True):
        ae = _model(cuda_device)
        ae.configure_optimizer()
        g = torch.randn(ae._flat_grad.shape, generator=torch.Generator().manual_seed(3)).to(cuda_device) * 1e-3
        if with_nan:
            ae._flat_grad.copy_(g)
            ae._flat_grad[777] = float("nan")
            ae.optimiser.step(max_norm=1.0, ema=ae.avg_params)
        ae._flat_grad.copy_(g)
        ae.optimiser.step(max_norm=1.0, ema=ae.avg_params)
        torch.cuda.synchronize()
        st = ae.optimiser.state_dict()
        runs.append(([t.detach().clone() for t in (ae._flat_param, ae.optimiser.exp_avg, ae.optimiser.exp_avg_sq,
                                                  ae.avg_params)], float(st["state"][0]["step"])))
    (ref, ref_step), (got, got_step) = runs
    assert ref_step == got_step == 1.0
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("runs", [(3, 9, 2), (1, 12, 3, 10, 1)])
def test_many_skipped_updates_keep_adams_step(cuda_device, runs):
    """Runs of consecutive non-finite steps with no settle (state_dict) in between, longer than the
    8-entry host table of bias corrections: the device skip count
    reaches 9..13, and every finite update after it must use Adam's bias correction of the updates
    actually applied.  runs = (finite, skipped, finite, ...): compared with torch.optim.Adam +
    clip_grad_norm_ + the EMA fed only the finite steps, and the step count after a settle."""
    n = 50_021
    torch.manual_seed(11)
    p0 = torch.randn(n)
    pr = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([pr], lr=1e-3, betas=(0.9, 0.999), eps=1e-8)
    ema_ref = p0.clone()
    p = p0.clone().to(cuda_device)
    m = torch.zeros(n, device=cuda_device)
    v = torch.zeros(n, device=cuda_device)
    ema = p.clone()
    skips = torch.zeros(1, dtype=torch.int32, device=cuda_device)
    norm = torch.empty((), device=cuda_device)
    calls = applied = 0
    for i, cnt in enumerate(runs):
        for _ in range(cnt):
            g = torch.randn(n) * 1e-2
            gd = g.to(cuda_device)
            if i % 2:
                gd[101] = float("nan")
            else:
                pr.grad = g.clone()
                torch.nn.utils.clip_grad_norm_([pr], max_norm=1.0)
                opt.step()
                ema_ref = 0.9999 * ema_ref + (1 - 0.9999) * pr.detach()
                applied += 1
            calls += 1
            _lib.call("avc_clip_adam_ema_dev", _lib.context(cuda_device), n, p.data_ptr(), gd.data_ptr(),
                      m.data_ptr(), v.data_ptr(), ema.data_ptr(), 1e-3, 0.9, 0.999, 1e-8, 0.0, calls, 1.0, 0.9999,
                      norm.data_ptr(), skips.data_ptr(), _lib.stream(cuda_device))
    torch.cuda.synchronize()
    assert calls - int(skips.item()) == applied
    assert (p.cpu() - pr.detach()).abs().max().item() < 2e-7 * max(1.0, pr.abs().max().item())
    assert (ema.cpu() - ema_ref).abs().max().item() < 4e-7 * max(1.0, ema_ref.abs().max().item())
    # the moments carry the clip coefficient c (fp64 norm here; torch's fp32 norm of 5e4 squares
    # is ~1e-5 relative off), m ~ c and v ~ c^2, while the update m / sqrt(v) cancels c -- hence the
    # tight bound on the parameters above and a c-sized one here.  (The bias corrections this test
    # is about enter the parameters only.)
    st = opt.state[pr]
    for got, ref in ((m.cpu(), st["exp_avg"]), (v.cpu(), st["exp_avg_sq"])):
        assert ((got - ref).abs() <= 1e-4 * ref.abs() + 1e-5 * ref.abs().max()).all()


def test_fused_adam_settles_after_many_skips(cuda_device):
    """FusedAdam (the module path): 10 NaN steps between finite ones, then state_dict(): the same
    parameters, moments, EMA and step count as the finite steps alone."""
    res = []
    for with_nan in (False, True):
        ae = _model(cuda_device)
        ae.configure_optimizer()
        gen = torch.Generator().manual_seed(5)
        gs = [torch.randn(ae._flat_grad.shape, generator=gen).to(cuda_device) * 1e-3 for _ in range(3)]
        for k, g in enumerate(gs):
            if with_nan and k > 0:
                for _ in range(10):
                    ae._flat_grad.copy_(g)
                    ae._flat_grad[4242] = float("inf")
                    ae.optimiser.step(max_norm=1.0, ema=ae.avg_params)
            ae._flat_grad.copy_(g)
            ae.optimiser.step(max_norm=1.0, ema=ae.avg_params)
        torch.cuda.synchronize()
        st = ae.optimiser.state_dict()
        res.append(([t.detach().clone() for t in (ae._flat_param, ae.optimiser.exp_avg, ae.optimiser.exp_avg_sq,
                                                 ae.avg_params)], float(st["state"][0]["step"])))
    (ref, ref_step), (got, got_step) = res
    assert ref_step == got_step == 3.0
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


def test_cooperative_launch_matches(cuda_device):
    """avc_lstm_persist_coop(1): the same kernels under hipLaunchCooperativeKernel (runtime
    co-residency guarantee), eager and graph-replayed, bit-identical to the default launch."""
    ae = _model(cuda_device)
    x, co, ct = _batch(cuda_device)
    with torch.no_grad():
        ref = [o.clone() for o in ae(x, co, ct)]
        _lib.call("avc_lstm_persist_coop", 1)
        try:
            runs = [[o.clone() for o in ae(x, co, ct)] for _ in range(3)]
            torch.cuda.synchronize()
        finally:
            _lib.call("avc_lstm_persist_coop", 0)
    for run in runs:
        for a, b in zip(run, ref):
            assert torch.equal(a, b)
    ae.check_health()


def test_alternating_launch_layouts(cuda_device):
    """One-layer persistent launches of different H at the same (T, batch groups) alternate on one
    context (decoder.lstm1 H=512 and the per-layer decoder.lstm2 H=1024 in training): each launch
    layout owns its counter region, so no epoch arithmetic leaks between them.  Outputs against
    the launch-per-step kernel (avc_lstm_persist_tune(0)), no give-ups."""
    from autovc_amd import ops
    T, B = 128, 64
    g = torch.Generator(device="cpu").manual_seed(3)
    layers = []
    for H, din in ((512, 320), (1024, 512)):
        w = [((torch.rand(4 * H, din, generator=g) - 0.5) * 0.1), ((torch.rand(4 * H, H, generator=g) - 0.5) * 0.1),
             torch.rand(4 * H, generator=g) * 0.1, torch.rand(4 * H, generator=g) * 0.1]
        layers.append(([t.to(cuda_device) for t in w], torch.rand(T * B, din, generator=g).to(cuda_device)))
    refs = []
    _lib.call("avc_lstm_persist_tune", 0)
    try:
        for w, x in layers:
            refs.append(ops.LSTMLayer.apply(x, *w, T, B, False))
    finally:
        _lib.call("avc_lstm_persist_tune", 2)
    before = _giveups()
    for _ in range(4):
        for (w, x), ref in zip(layers, refs):
            for save in (False, True):
                y = ops.LSTMLayer.apply(x, *w, T, B, save)
                assert float((y - ref).abs().max()) <= 1e-6
    assert _giveups() == before


def test_persistent_bptt_timeout_is_nan_and_next_call_raises(cuda_device):
    """The persistent BPTT (bptt_persist_kernel, B = 128) under the same safety net: an injected
    give-up leaves NaN gradients (never plausible numbers), and the next persistent launch on the
    context raises after resetting the counter state; then the layer runs normally again."""
    from autovc_amd import ops
    B, T, H, din = 128, 8, 1024, 512
    g = torch.Generator().manual_seed(9)
    k = 1.0 / H ** 0.5
    ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(cuda_device).requires_grad_(True)
          for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    x = (torch.randn(T * B, din, generator=g) * 0.5).to(cuda_device).requires_grad_(True)
    dy = torch.randn(T * B, H, generator=g).to(cuda_device)
    y = ops.LSTMLayer.apply(x, *ws, T, B, True)
    torch.cuda.synchronize()
    before = _giveups()
    _lib.call("avc_debug_persist_inject", 1)  # the next persistent launch: the BPTT
    y.backward(dy)
    torch.cuda.synchronize()
    assert _giveups() > before, "the injected BPTT launch did not give up"
    assert torch.isnan(ws[1].grad).any() and torch.isnan(x.grad).any()
    with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
        ops.LSTMLayer.apply(x, *ws, T, B, True)
    for w in ws:
        w.grad = None
    x.grad = None
    y = ops.LSTMLayer.apply(x, *ws, T, B, True)
    y.backward(dy)
    torch.cuda.synchronize()
    assert all(torch.isfinite(w.grad).all() for w in ws) and torch.isfinite(x.grad).all()
