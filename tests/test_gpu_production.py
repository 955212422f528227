"""Parity at the production sizes of BASELINE.json: C2 (B = 64, T = 128 forward) and C3 (B = 256,
T = 128 training step).  The golden fixtures are B <= 3, where several kernels take other plans
(fp32 fallback GEMM for rows that are not whole 16/32-row fragment tiles, other LSTM tile and
batch-group configurations); these tests pin the plans the bench actually runs against the CPU
oracle (oracle/autovc_oracle.py, itself pinned to the reference's outputs by tests/golden).

Tolerances (BASELINE north_star): max|d| <= 1e-4 on mel / mel_post / codes; BN running buffers
1e-5; training: see each test."""
import numpy as np
import pytest
import torch

from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import onehot_embedding, synthetic_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu

TOL_MEL = 1e-4


def _model(dev, train=True, seed=0):
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(torch_state_dict(seed))
    ae.to(dev)
    ae.train(train)
    return ae


def _threads():
    torch.set_num_threads(min(16, torch.get_num_threads()))


@pytest.fixture(scope="module")
def c2_case():
    """The bench's C2 batch (bench.py setup_generator, rank 0) and the oracle's answer for it in
    both BatchNorm modes."""
    from oracle import autovc_oracle as orc
    _threads()
    B, T = 64, 128
    x = synthetic_mel(1, B, T)
    co, ct = synthetic_embedding(101, B), synthetic_embedding(201, B)
    sd = torch_state_dict(0)
    ref = {}
    with torch.no_grad():
        for train in (True, False):
            bufs = {k: v.clone() for k, v in sd.items() if "running" in k or "num_batches" in k}
            out = orc.forward(sd, torch.from_numpy(x), torch.from_numpy(co), torch.from_numpy(ct), train, bufs)
            ref[train] = (out, bufs)
    return x, co, ct, ref


@pytest.mark.parametrize("train", [True, False], ids=["train_bn", "eval_bn"])
@pytest.mark.parametrize("path", ["fused", "autograd", "layers"])
def test_c2_forward_against_oracle(cuda_device, c2_case, path, train):
    """C2 forward through each host path: fused (no_grad, as bench.py), autograd (grad enabled,
    the call convert() makes: voice_converter.py:172-174) and the per-layer path (training)."""
    x, co, ct, ref = c2_case
    ae = _model(cuda_device, train)
    ae.fused_autograd = path != "layers"
    xg, cog, ctg = (torch.from_numpy(a).to(cuda_device) for a in (x, co, ct))
    if path == "fused":
        with torch.no_grad():
            outs = ae(xg, cog, ctg)
    else:
        outs = ae(xg, cog, ctg)
        assert outs[1].requires_grad
    torch.cuda.synchronize()
    (rm, rp, rc), bufs = ref[train]
    errs = [float((o.detach().cpu() - r).abs().max()) for o, r in zip(outs, (rm, rp, rc))]
    print(f"C2 {path} {'train' if train else 'eval'}-BN: max|d| mel {errs[0]:.2e} mel_post {errs[1]:.2e} "
          f"codes {errs[2]:.2e}")
    assert max(errs) <= TOL_MEL
    for k, v in ae.state_dict().items():
        if k in bufs:
            if k.endswith("num_batches_tracked"):
                assert int(v) == int(bufs[k]), k
            else:
                assert float((v.cpu() - bufs[k]).abs().max()) <= 1e-5, k


def test_c2_grad_enabled_backward_matches_layers(cuda_device, c2_case):
    """The grad-enabled fused node back-propagates through a per-layer recompute: gradients of a
    fixed projection of (mel, mel_post, codes) w.r.t. parameters and inputs equal the per-layer
    path's, and the BN running buffers move once per forward (not again in the recompute)."""
    x, co, ct, _ = c2_case
    res = {}
    for path in ("autograd", "layers"):
        ae = _model(cuda_device, True)
        ae.fused_autograd = path == "autograd"
        xg = torch.from_numpy(x).to(cuda_device).requires_grad_(True)
        cog = torch.from_numpy(co).to(cuda_device).requires_grad_(True)
        ctg = torch.from_numpy(ct).to(cuda_device)
        mel, post, codes = ae(xg, cog, ctg)
        g = torch.Generator(device="cpu").manual_seed(5)
        wm, wp = (torch.rand(mel.shape, generator=g).to(cuda_device) for _ in range(2))
        wc = torch.rand(codes.shape, generator=g).to(cuda_device)
        ((mel * wm).sum() + (post * wp).sum() + (codes * wc).sum()).backward()
        torch.cuda.synchronize()
        res[path] = ({k: p.grad.detach().cpu().clone() for k, p in ae.named_parameters()},
                     xg.grad.cpu(), cog.grad.cpu(),
                     {k: v.cpu().clone() for k, v in ae.state_dict().items() if "running" in k or "num_b" in k})
    ga, gl = res["autograd"], res["layers"]
    for k in ga[0]:
        d = float((ga[0][k] - gl[0][k]).abs().max())
        scale = float(gl[0][k].abs().max()) + 1e-30
        assert d <= 1e-5 * scale, f"{k}: max|d grad| {d:.3e} (scale {scale:.3e})"
    for a, b in ((ga[1], gl[1]), (ga[2], gl[2])):
        assert float((a - b).abs().max()) <= 1e-5 * (float(b.abs().max()) + 1e-30)
    for k in ga[3]:
        assert torch.allclose(ga[3][k].double(), gl[3][k].double(), atol=1e-6, rtol=0), k


@pytest.fixture(scope="module")
def c3_case():
    """C3: the bench's training batch (B = 256, T = 128, one-hot speaker ids) and the oracle's
    loss and parameter gradients for it (fp32 CPU autograd of the reference loss, model.py:184-215)."""
    from oracle import autovc_oracle as orc
    _threads()
    B, T = 256, 128
    X = torch.from_numpy(synthetic_mel(1, B, T))
    c = torch.from_numpy(onehot_embedding(B))
    sd = torch_state_dict(0)
    tr = orc.Trainer(sd)
    sdc = tr.sd()
    od, op, oc = orc.forward(sdc, X, c, c, True, tr.bufs)
    loss = orc.loss_fn(sdc, X, c, od, op, oc, tr.bufs)
    grads = dict(zip(tr.names, torch.autograd.grad(loss, [tr.p[k] for k in tr.names])))
    norm = float(torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads.values()])))
    # the same in float64: how far the fp32 reference itself sits from exact arithmetic
    tr64 = orc.Trainer({k: v.double() for k, v in sd.items()})
    s64 = tr64.sd()
    od, op, oc = orc.forward(s64, X.double(), c.double(), c.double(), True, tr64.bufs)
    l64 = orc.loss_fn(s64, X.double(), c.double(), od, op, oc, tr64.bufs)
    g64 = dict(zip(tr64.names, torch.autograd.grad(l64, [tr64.p[k] for k in tr64.names])))
    return X, c, float(loss.detach()), grads, norm, g64


def _gpu_grads(dev, X, c, gemm_mode=None):
    from autovc_amd import _lib
    if gemm_mode is not None:
        _lib.call("avc_gemm_tune", gemm_mode)
    try:
        ae = _model(dev)
        Xg, cg = X.to(dev), c.to(dev)
        md, mp, mc = ae._forward_layers(Xg, cg, cg)
        loss = ae._loss(Xg, cg, md, mp, mc)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        if gemm_mode is not None:
            _lib.call("avc_gemm_tune", 2)
    return loss.item(), {k: p.grad.detach().cpu().double() for k, p in ae.named_parameters()}


def test_c3_gradients_against_oracle(cuda_device, c3_case):
    """C3 backward at its production plan (long-K weight gradients on 128x128 tiles with split-K,
    scaled 3xf16 products everywhere).  As at B = 32 (test_gpu_model.py::
    test_gradients_split_backward_path) the loss is not smooth in the weights (L1 signs, ReLU
    masks), so the backward arithmetic is isolated by re-running the SAME forward with the
    backward products on the compensated fp32 kernel (avc_gemm_tune(3)): <= 2e-5 relative L2 per
    tensor.  Against the fp32 CPU oracle: loss 1e-5 relative, every gradient <= 5e-3 relative L2
    (reported), the total gradient norm 1e-3 relative.  Sign flips of clearly non-zero gradient
    elements against float64 (what Adam's first step acts on) at most twice the fp32 CPU
    oracle's own count."""
    X, c, loss_ref, g_ref, norm_ref, g64 = c3_case
    l16, g16 = _gpu_grads(cuda_device, X, c)
    l32, g32 = _gpu_grads(cuda_device, X, c, 3)
    assert l16 == l32
    assert l16 == pytest.approx(loss_ref, rel=1e-5)
    norm = float(torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in g16.values()])))
    worst_a, worst_t = (0.0, ""), (0.0, "")
    for k, b in g_ref.items():
        b = b.double()
        if k.endswith(".0.conv.bias"):  # exactly-zero true gradient (train-mode BN follows)
            assert g16[k].norm().item() < 1e-5, k
            continue
        d = ((g16[k] - g32[k]).norm() / g32[k].norm()).item()
        t = ((g16[k] - b).norm() / b.norm()).item()
        worst_a, worst_t = max(worst_a, (d, k)), max(worst_t, (t, k))
        assert d < 2e-5, f"{k}: split vs fp32 backward products differ by {d:.2e}"
        assert t < 5e-3, f"{k}: {t:.2e} from the fp32 CPU oracle"
    # Adam's first step is ~lr*sign(g): count gradient elements whose sign differs from exact
    # (float64) arithmetic, among those clearly above noise (|g64| > 0.1 of the tensor's RMS), for
    # this path and for the fp32 reference itself
    flips_gpu = flips_ref = n_clear = 0
    for k, e in g64.items():
        m = e.abs() > 0.1 * e.pow(2).mean().sqrt()
        n_clear += int(m.sum())
        flips_gpu += int(((torch.sign(g16[k]) != torch.sign(e)) & m).sum())
        flips_ref += int(((torch.sign(g_ref[k].double()) != torch.sign(e)) & m).sum())
    print(f"C3 sign flips vs float64 among {n_clear} clearly-signed gradient elements: "
          f"HIP {flips_gpu}, fp32 CPU oracle {flips_ref}")
    assert flips_gpu <= 2 * flips_ref + 100
    print(f"C3 loss {l16:.7f} (oracle {loss_ref:.7f}); grad norm {norm:.6f} (oracle {norm_ref:.6f}); "
          f"split vs fp32 products worst {worst_a[0]:.2e} ({worst_a[1]}); vs oracle worst {worst_t[0]:.2e} "
          f"({worst_t[1]})")
    assert norm == pytest.approx(norm_ref, rel=1e-3)


def test_c3_train_step_against_oracle(cuda_device, c3_case):
    """One full C3 train_step (forward, loss, backward, fused clip 1.0 + Adam + EMA) from identical
    parameters against the oracle Trainer (model.py:303-321).  Loss and pre-clip grad norm as in
    test_c3_gradients_against_oracle.  Adam's first step moves every element by ~lr*sign(g): the
    update may flip only where |g| is at rounding-noise level, so every element stays within
    2*lr*1.01 of the oracle's, >= 98 % of all elements agree to 1e-6 (measured 98.74 %: the rest
    are elements whose gradient is at rounding level), and the EMA sums agree to 1e-6 relative."""
    from oracle import autovc_oracle as orc
    X, c, loss_ref, _, norm_ref, _ = c3_case
    ae = _model(cuda_device)
    ae.configure_optimizer()
    loss, norm = ae.train_step(X.to(cuda_device), c.to(cuda_device))
    torch.cuda.synchronize()
    tr = orc.Trainer(torch_state_dict(0))
    l_o, n_o = tr.step(X, c)
    assert l_o == pytest.approx(loss_ref, rel=1e-6) and n_o == pytest.approx(norm_ref, rel=1e-6)
    assert loss.item() == pytest.approx(l_o, rel=1e-5)
    assert norm.item() == pytest.approx(n_o, rel=1e-3)
    # The first Adam step is lr * g / (|g| + eps) ~ lr * sign(g): where the gradient's sign is
    # decided by rounding (test_c3_gradients_against_oracle counts those against float64 for
    # both implementations) the two updates differ by 2*lr; everywhere else they agree.
    worst = 0.0
    agree = total = 0
    for k, p in ae.named_parameters():
        d = (p.detach().cpu().double() - tr.p[k].detach().double()).abs()
        worst = max(worst, float(d.max()))
        agree += int((d <= 1e-6).sum())
        total += d.numel()
    ema_d = abs(float(ae.avg_params.double().sum()) - float(tr.avg.double().sum()))
    print(f"C3 train_step: loss {loss.item():.7f} (oracle {l_o:.7f}), norm {norm.item():.6f} (oracle {n_o:.6f}); "
          f"worst |d param| {worst:.2e}; params agreeing to 1e-6: {100 * agree / total:.3f} %; "
          f"|d EMA sum| {ema_d:.2e}")
    assert worst <= 2 * 1e-3 * 1.01
    assert agree >= 0.98 * total
    assert ema_d <= 1e-6 * float(tr.avg.double().abs().sum())
