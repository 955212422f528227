"""The conv forward handing its weight gradient the split of x (avc_conv_bn_act_forward_wg /
avc_conv_bn_act_backward_wg, round 6): a conv -> conv chain of the per-layer training path
(encoder.py:69-70; the second conv's x carries the first one's max words) gives bit-identical
outputs and gradients with and without the image, and the gradients match fp64 autograd."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from autovc_amd import ops

pytestmark = pytest.mark.gpu


def _chain(dev, params, x, T, B):
    W0, b0, g0, be0, W1, b1, g1, be1 = params
    h = ops.ConvBNAct.apply(x, W0, b0, g0, be0, None, None, True, 0.1, 1e-5, ops.ACT_RELU, None, T, B)
    return ops.ConvBNAct.apply(h, W1, b1, g1, be1, None, None, True, 0.1, 1e-5, ops.ACT_RELU, None, T, B)


@pytest.mark.parametrize("T,B,cin,c,img", [(64, 64, 512, 512, True), (32, 32, 256, 128, True), (20, 8, 128, 64, False)])
def test_wgrad_image_bit_identical(cuda_device, T, B, cin, c, img):
    g = torch.Generator().manual_seed(T + B + c)
    shapes = [(c, cin, 5), (c,), (c,), (c,), (c, c, 5), (c,), (c,), (c,)]
    host = []
    for i, sh in enumerate(shapes):
        if len(sh) == 3:
            host.append((torch.rand(*sh, generator=g) - 0.5) * (2.0 / np.sqrt(sh[1] * 5)))
        elif i in (2, 6):
            host.append(torch.rand(*sh, generator=g) + 0.5)
        else:
            host.append((torch.rand(*sh, generator=g) - 0.5) * 0.2)
    xh = torch.rand(T * B, cin, generator=g)
    dyh = torch.randn(T * B, c, generator=g)
    assert (ops.wgrad_image_bytes(T, B, c, c) > 0) == img  # (B = 8: taps are not 32-row shifts)
    runs = []
    for use in (True, False):
        old = ops._WGRAD_IMAGE
        ops._WGRAD_IMAGE = use
        try:
            params = [p.to(cuda_device).requires_grad_(True) for p in host]
            x = xh.to(cuda_device).requires_grad_(True)
            y = _chain(cuda_device, params, x, T, B)
            y.backward(dyh.to(cuda_device))
            torch.cuda.synchronize()
            runs.append([y.detach().cpu(), x.grad.cpu()] + [p.grad.cpu() for p in params])
        finally:
            ops._WGRAD_IMAGE = old
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    # and against fp64 autograd of the same chain
    P = [p.double().requires_grad_(True) for p in host]
    xd = xh.double().requires_grad_(True)

    def layer(h, W, b, gm, bt):
        z = F.conv1d(h.reshape(T, B, -1).permute(1, 2, 0), W, b, padding=2)
        z = F.batch_norm(z, None, None, gm, bt, training=True, eps=1e-5)
        return torch.relu(z).permute(2, 0, 1).reshape(T * B, -1)

    yd = layer(layer(xd, *P[:4]), *P[4:])
    yd.backward(dyh.double())
    got = runs[0]
    assert (got[0].double() - yd.detach()).abs().max().item() < 1e-4
    # (the conv biases are left out: under train-mode BN their true gradient is 0 and the fp32 sum
    # over T*B rows is rounding noise; the bit-identity above covers them)
    for i, (gg, ref) in enumerate(zip(got[2:], [p.grad for p in P])):
        if i in (1, 5):
            continue
        err = (gg.double() - ref).abs().max().item()
        assert err <= 2e-4 * max(1.0, ref.abs().max().item()), (i, err)
    err = (got[1].double() - xd.grad).abs().max().item()
    assert err <= 2e-4 * max(1.0, xd.grad.abs().max().item()), err
