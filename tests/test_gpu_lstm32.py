"""The encoder BiLSTM (H = 32) forward with its memory operations on a second wave
(lstm32_fwd2_kernel, avc_lstm32_tune(1), round 5) against the one-wave kernel (avc_lstm32_tune(4)):
the same step expressions in the same order, so outputs, saved gates / cell states (through the
backward's gradients) and every gradient must agree bit for bit -- ragged T (a partial last group
of 8 steps), inference and training.  Reference layer: autovc/auto_encoder/encoder.py:51,73."""
import pytest
import torch

from autovc_amd import _lib, ops

pytestmark = pytest.mark.gpu


def _run(dev, T, B, din, save, mode, seed=3):
    g = torch.Generator().manual_seed(seed + T + B)
    H = 32
    ws = [((torch.rand(*s, generator=g) * 2 - 1) * 0.3).to(dev).requires_grad_(save)
          for s in [(128, din), (128, H), (128,), (128,)] * 2]
    x = torch.randn(T * B, din, generator=g).to(dev).requires_grad_(save)
    dy = torch.randn(T * B, 2 * H, generator=g).to(dev)
    _lib.call("avc_lstm32_tune", mode)
    try:
        y = ops.BiLSTMLayer.apply(x, *ws, T, B, save)
        out = [y.detach().clone()]
        if save:
            y.backward(dy)
            out += [x.grad.clone()] + [w.grad.clone() for w in ws]
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_lstm32_tune", 1)
    return out


@pytest.mark.parametrize("T,B,din,save", [(128, 64, 336, False), (13, 5, 64, True), (1000, 3, 64, True),
                                          (128, 256, 336, True), (1, 2, 64, True), (9, 1, 64, False)])
def test_two_wave_forward_is_bit_identical(cuda_device, T, B, din, save):
    new = _run(cuda_device, T, B, din, save, 1)
    old = _run(cuda_device, T, B, din, save, 4)
    for i, (a, b) in enumerate(zip(new, old)):
        assert torch.isfinite(a).all(), i
        assert torch.equal(a, b), f"output {i}: max|d| {(a - b).abs().max().item():.3e}"
