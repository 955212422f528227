"""Persistent BPTT with the unit-group-fast epilogue mapping (avc_bptt_coalesce(1))
against the round-3 row-fast mapping (avc_bptt_coalesce(0)).

Only the thread <-> (row, unit group) assignment of phase B changes, plus the LDS staging of the
split dG it hands to the next step and the order in which the bias gradients' column sums are
combined.  Every dG element is formed by the same expression from the same partial sums in the
same order, so dX, dW_ih and dW_hh must agree bit for bit; the biases within rounding of a
different summation order.  Shapes: the three persistent instances (B = 256 / H = 1024: 16
K-slices; B = 128 / H = 1024 and B = 256 / H = 512: 32).  Reference: decoder.py:37,53."""
import pytest
import torch

from autovc_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEFAULT = 1  # the library's default (avc_bptt_coalesce)


def _bwd(dev, B, T, din, H, mode):
    g = torch.Generator().manual_seed(B + H + din)
    k = 1.0 / H ** 0.5
    ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev).requires_grad_(True)
          for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    x = (torch.randn(T * B, din, generator=g) * 0.5).to(dev).requires_grad_(True)
    dy = torch.randn(T * B, H, generator=g).to(dev)
    _lib.call("avc_bptt_coalesce", mode)
    try:
        launches = _lib.persist_launches(dev)
        y = ops.LSTMLayer.apply(x, *ws, T, B, True)
        y.backward(dy)
        torch.cuda.synchronize()
        persistent = _lib.persist_launches(dev) - launches
    finally:
        _lib.call("avc_bptt_coalesce", DEFAULT)
    return [x.grad.clone()] + [w.grad.clone() for w in ws], persistent


@pytest.mark.parametrize("B,T,din,H", [(256, 48, 512, 1024), (128, 40, 1024, 1024), (256, 40, 320, 512)])
def test_coalesced_epilogue_is_bit_identical(cuda_device, B, T, din, H):
    new, n1 = _bwd(cuda_device, B, T, din, H, 1)
    old, n0 = _bwd(cuda_device, B, T, din, H, 0)
    assert n1 >= 1 and n0 == n1  # the persistent BPTT ran in both
    for name, a, b in zip(["dx", "dW_ih", "dW_hh", "db_ih", "db_hh"], new, old):
        d = float((a.double() - b.double()).abs().max())
        print(f"B={B} H={H} {name}: max |d| {d:.2e} (max |g| {float(b.abs().max()):.2e})")
        if name.startswith("db"):
            assert d <= 1e-6 * max(1.0, float(b.abs().max())), name
        else:
            assert torch.equal(a, b), name
