"""Conv1d + BatchNorm backward with dY written already split by the BatchNorm backward
(avc_bn_bwd_frag) against the fp32-dY path (avc_bn_bwd_frag(0)) and float64 autograd.

The split-writing pass scales dY by the power of two of a proven upper bound on max |dY|
(bn_bwd_final_kernel, BnBound) instead of the exact max.  A power-of-two scale moves every element
by the same number of binades, so hi / lo -- and every 3xf16 product, unscaled exactly -- are
unchanged for all elements that stay normal in f16; only elements ~2^-27 below the operand's max
can round differently.  So dX and dW must agree with the fp32-dY path to within a few ulps of
their magnitudes (almost every element bit for bit), d_gamma / d_beta bit for bit (same reduce
pass), and everything must hold over gradient magnitudes from 1e-8 to 1e6 (the bound only works
if it tracks the scale).  Batches are multiples of 16 so both products stream fragments.
Reference layers: autovc/auto_encoder/encoder.py:69-70, decoder.py:69-71, postnet.py:50-63."""
import pytest
import torch
import torch.nn.functional as F

from autovc_amd import _lib, ops

pytestmark = pytest.mark.gpu

DEFAULT = 1  # the library's default (avc_bn_bwd_frag)
CASES = [(16, 64, 336, 512, ops.ACT_RELU, True, False), (32, 40, 512, 512, ops.ACT_TANH, True, False),
         (16, 48, 512, 80, ops.ACT_NONE, True, True), (16, 64, 80, 512, ops.ACT_TANH, False, False)]


def _t(a, dev):
    return torch.as_tensor(a, dtype=torch.float32).to(dev).contiguous()


def _grads(dev, B, T, cin, cout, act, training, res, dscale, mode, mean_dom=0.0):
    g = torch.Generator().manual_seed(B * 1000 + T + cin + cout)
    x = torch.rand(B, cin, T, generator=g)
    W = (torch.rand(cout, cin, 5, generator=g) - 0.5) * 0.1
    bias = (torch.rand(cout, generator=g) - 0.5) * 0.1
    gamma = torch.rand(cout, generator=g) + 0.5
    beta = (torch.rand(cout, generator=g) - 0.5) * 0.4
    rm = (torch.rand(cout, generator=g) - 0.5) * 0.2
    rv = torch.rand(cout, generator=g) + 0.5
    resid = torch.randn(B, cout, T, generator=g) if res else None
    dout = torch.randn(B, cout, T, generator=g) * dscale
    if mean_dom:  # a gradient that is mostly its channel mean: c (1 + mean_dom * noise)
        dout = dscale * (3.0 + 3.0 * mean_dom * torch.randn(B, cout, T, generator=g))
    fr = x.permute(2, 0, 1).reshape(T * B, cin)
    xg = _t(fr, dev).requires_grad_(True)
    pg = [_t(t, dev).requires_grad_(True) for t in (W, bias, gamma, beta)]
    rg = _t(resid.permute(2, 0, 1).reshape(T * B, cout), dev) if res else None
    _lib.call("avc_bn_bwd_frag", mode)
    try:
        out = ops.ConvBNAct.apply(xg, *pg, _t(rm, dev), _t(rv, dev), training, 0.1, 1e-5, act, rg, T, B)
        out.backward(_t(dout.permute(2, 0, 1).reshape(T * B, cout), dev))
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_bn_bwd_frag", DEFAULT)
    got = [xg.grad.cpu()] + [p.grad.cpu() for p in pg]
    # float64 autograd of the same layer
    params = [t.double().clone().requires_grad_(True) for t in (x, W, bias, gamma, beta)]
    y = F.batch_norm(F.conv1d(params[0], params[1], params[2], padding=2), rm.double().clone(),
                     rv.double().clone(), params[3], params[4], training=training, momentum=0.1, eps=1e-5)
    y = {ops.ACT_RELU: torch.relu, ops.ACT_TANH: torch.tanh, ops.ACT_NONE: lambda v: v}[act](y)
    if res:
        y = y + resid.double()
    y.backward(dout.double())
    ref = [params[0].grad.permute(2, 0, 1).reshape(T * B, cin)] + [p.grad for p in params[1:]]
    return got, ref


@pytest.mark.parametrize("dscale", [1.0, 1e-8, 1e6])
@pytest.mark.parametrize("B,T,cin,cout,act,training,res", CASES)
def test_split_writing_bn_backward_matches_fp32_path(cuda_device, B, T, cin, cout, act, training, res, dscale):
    new, ref64 = _grads(cuda_device, B, T, cin, cout, act, training, res, dscale, 1)
    old, _ = _grads(cuda_device, B, T, cin, cout, act, training, res, dscale, 0)
    names = ["dx", "dW", "dbias", "dgamma", "dbeta"]
    for name, a, b, r in zip(names, new, old, ref64):
        # (train mode: the exact bias gradient is 0, so its noise is measured against d_beta's scale)
        scale = float((ref64[4] if name == "dbias" and training else r).abs().max()) or 1.0
        d_old = float((a.double() - b.double()).abs().max()) / scale
        d_f64 = float((a.double() - r).abs().max()) / scale
        same = float((a == b).double().mean())
        print(f"{name}: |new - fp32-dY path| {d_old:.2e}, |new - f64| {d_f64:.2e} (rel. to max), "
              f"bit-identical {100 * same:.2f} %")
        assert torch.isfinite(a).all(), name
        if name in ("dgamma", "dbeta"):
            assert torch.equal(a, b), name  # the same reduce pass
        elif name == "dbias":
            if training:  # exactly 0 in exact arithmetic (BN removes it): rounding noise only
                assert d_f64 < 1e-3 and d_old < 1e-3, name
            else:
                assert d_old < 1e-6 and d_f64 < 3e-5, name
        else:
            assert d_old < 1e-6, name
            assert same > 0.98, name
            assert d_f64 < (2e-5 if name == "dx" else 3e-5), name


@pytest.mark.parametrize("mean_dom", [1e-3, 1e-5])
@pytest.mark.parametrize("B,T,cin,cout,act,training,res", [CASES[2], (16, 64, 512, 512, ops.ACT_NONE, True, False)])
def test_mean_dominated_gradient_keeps_the_bound_tight(cuda_device, B, T, cin, cout, act, training, res, mean_dom):
    """dY = g is (dA - k1 - x^ k2) cancels when dA is mostly its channel mean k1.  A bound
    built from max|dA| + |k1| then sits log2(1 / mean_dom) binades above the true max |dY|, and every
    element drops that far toward f16's subnormals.  The bound now takes the signed range of dA about
    k1, so the split-writing path stays bit-identical to the fp32-dY path here as well."""
    new, ref64 = _grads(cuda_device, B, T, cin, cout, act, training, res, 1.0, 1, mean_dom)
    old, _ = _grads(cuda_device, B, T, cin, cout, act, training, res, 1.0, 0, mean_dom)
    for name, a, b, r in zip(["dx", "dW"], new[:2], old[:2], ref64[:2]):
        scale = float(r.abs().max()) or 1.0
        d_old = float((a.double() - b.double()).abs().max()) / scale
        same = float((a == b).double().mean())
        print(f"mean_dom {mean_dom:g} {name}: |new - fp32-dY path| {d_old:.2e} (rel. to max), bit-identical {100 * same:.2f} %")
        assert torch.isfinite(a).all(), name
        assert d_old < 1e-6 and same > 0.98, name
