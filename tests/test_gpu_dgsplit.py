"""The LSTM backward's one-pass split of dG into both operand images (avc_dg_dual_split(1),
split_frag32_dual_kernel) against two split passes (avc_dg_dual_split(0)).

Each image element is scaled and split by the expressions split_frag32_kernel uses, so dX and the
weight gradients must agree bit for bit.  Shapes: the persistent-BPTT instances (decoder lstm2 /
lstm1 at the C3 batch) and a launch-per-step one.  Reference: decoder.py:37,53,65,74."""
import pytest
import torch

from autovc_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEFAULT = 1  # the library's default (avc_dg_dual_split)


def _bwd(dev, B, T, din, H, mode):
    g = torch.Generator().manual_seed(B + H + din + 7)
    k = 1.0 / H ** 0.5
    ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev).requires_grad_(True)
          for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    x = (torch.randn(T * B, din, generator=g) * 0.5).to(dev).requires_grad_(True)
    dy = torch.randn(T * B, H, generator=g).to(dev)
    _lib.call("avc_dg_dual_split", mode)
    try:
        y = ops.LSTMLayer.apply(x, *ws, T, B, True)
        y.backward(dy)
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_dg_dual_split", DEFAULT)
    return [x.grad.clone()] + [w.grad.clone() for w in ws]


@pytest.mark.parametrize("B,T,din,H", [(256, 24, 512, 1024), (256, 24, 320, 512), (64, 20, 512, 512)])
def test_dual_split_is_bit_identical(cuda_device, B, T, din, H):
    new = _bwd(cuda_device, B, T, din, H, 1)
    old = _bwd(cuda_device, B, T, din, H, 0)
    for name, a, b in zip(["dx", "dW_ih", "dW_hh", "db_ih", "db_hh"], new, old):
        d = float((a - b).abs().max())
        print(f"B={B} H={H} {name}: max |d| {d:.2e} (max |g| {float(b.abs().max()):.2e})")
        assert torch.isfinite(a).all(), name
        assert torch.equal(a, b), name
