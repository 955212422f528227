"""XCD-local BPTT of an H = 512 layer (bptt_xl_kernel, avc_bptt_xcd(1), round 5) against the
128-row-tile persistent BPTT (avc_bptt_xcd(0), bptt_persist_kernel<4, 32, 32, true>).

Groups of 32 batch rows run on one XCD each, with the whole split W_hh^T in their LDS; a
workgroup owns one 64-column K-slice for both phases, so its split dG never leaves the CU and the
only hand-off per step is the partials', inside the XCD.  The products (chunks, MFMA order), the
per-(row, K-slice) split scales, the partial order and the epilogue are the 128-row form's, so
dX, dW_ih, dW_hh and both bias gradients must agree bit for bit.  Reference layer: decoder.lstm1
(autovc/auto_encoder/decoder.py:37,65)."""
import ctypes

import pytest
import torch

from autovc_amd import _lib, ops

pytestmark = pytest.mark.gpu


def _giveups():
    n = ctypes.c_long(0)
    _lib.call("avc_lstm_persist_status", ctypes.byref(n))
    return n.value


def _layer(dev, B, T, din, H, seed):
    g = torch.Generator().manual_seed(seed)
    k = 1.0 / H ** 0.5
    ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev).requires_grad_(True)
          for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    x = (torch.randn(T * B, din, generator=g) * 0.5).to(dev).requires_grad_(True)
    dy = torch.randn(T * B, H, generator=g).to(dev)
    return ws, x, dy


def _bwd(dev, B, T, din, H, mode, seed=0):
    ws, x, dy = _layer(dev, B, T, din, H, seed)
    _lib.call("avc_bptt_xcd", mode)
    try:
        launches = _lib.persist_launches(dev)
        y = ops.LSTMLayer.apply(x, *ws, T, B, True)
        y.backward(dy)
        torch.cuda.synchronize()
        persistent = _lib.persist_launches(dev) - launches
    finally:
        _lib.call("avc_bptt_xcd", 1)  # (the default)
    return [x.grad.clone()] + [w.grad.clone() for w in ws], persistent


@pytest.mark.parametrize("B,T,din", [(256, 128, 320), (256, 40, 320), (256, 2, 320), (256, 3, 512)])
def test_xcd_local_bptt_is_bit_identical(cuda_device, B, T, din):
    H = 512
    before = _giveups()
    _lib.call("avc_debug_xl_census", (ctypes.c_uint * 2)())  # (clear)
    new, n1 = _bwd(cuda_device, B, T, din, H, 1, seed=B + T)
    seen = (ctypes.c_uint * 2)()
    _lib.call("avc_debug_xl_census", seen)
    old, n0 = _bwd(cuda_device, B, T, din, H, 0, seed=B + T)
    assert n1 >= 1 and n0 == n1  # the persistent BPTT ran in both
    print(f"B={B} T={T}: BPTT workgroups on a local group {seen[0]}, not local {seen[1]}")
    for name, a, b in zip(["dx", "dW_ih", "dW_hh", "db_ih", "db_hh"], new, old):
        assert torch.isfinite(a).all(), name
        assert torch.equal(a, b), f"{name}: max |d| {float((a.double() - b.double()).abs().max()):.2e}"
    assert _giveups() == before


@pytest.mark.parametrize("B,T", [(32, 64), (64, 48), (128, 40), (96, 5)])
def test_xcd_local_bptt_other_batches(cuda_device, B, T):
    """Batches the 128-row form does not take (avc_bptt_xcd(2); by default they keep the launch-per-
    step BPTT): the XCD-local form against that path (fp32 MFMA products) within the products'
    rounding."""
    H, din = 512, 320
    _lib.call("avc_debug_xl_census", (ctypes.c_uint * 2)())  # (clear)
    new, n1 = _bwd(cuda_device, B, T, din, H, 2, seed=B + T)
    seen = (ctypes.c_uint * 2)()
    _lib.call("avc_debug_xl_census", seen)
    old, n0 = _bwd(cuda_device, B, T, din, H, 1, seed=B + T)  # (the default: the step kernels)
    assert n1 == n0 + 1  # the XCD-local BPTT is the one extra persistent launch
    print(f"B={B} T={T}: BPTT workgroups on a local group {seen[0]}, not local {seen[1]}")
    for name, a, b in zip(["dx", "dW_ih", "dW_hh", "db_ih", "db_hh"], new, old):
        d = float((a.double() - b.double()).abs().max())
        m = float(b.abs().max())
        print(f"  {name}: max |d| {d:.2e} (max |g| {m:.2e})")
        assert torch.isfinite(a).all() and d <= 2e-5 * m + 1e-7, name


def test_xcd_local_bptt_repeated_launches(cuda_device):
    """Back-to-back launches on one counter region (the tags carry the launch epoch)."""
    B, T, din, H = 256, 24, 320, 512
    ref, _ = _bwd(cuda_device, B, T, din, H, 0, seed=5)
    for _ in range(4):
        got, _ = _bwd(cuda_device, B, T, din, H, 1, seed=5)
        for a, b in zip(got, ref):
            assert torch.equal(a, b)


def test_xcd_local_bptt_timeout_is_nan_and_next_call_raises(cuda_device):
    B, T, H, din = 256, 8, 512, 320
    ws, x, dy = _layer(cuda_device, B, T, din, H, 11)
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


def test_xcd_local_bptt_fallback_is_bit_identical(cuda_device):
    """Groups found not to share one XCD (forced here: avc_debug_xl_force_remote) hand the partials
    over with write-through stores and a counter per (step, group) instead -- the same bits."""
    B, T, din, H = 256, 40, 320, 512
    ref, _ = _bwd(cuda_device, B, T, din, H, 0, seed=7)
    _lib.call("avc_debug_xl_census", (ctypes.c_uint * 2)())  # (clear)
    _lib.call("avc_debug_xl_force_remote", 1)
    try:
        got, _ = _bwd(cuda_device, B, T, din, H, 1, seed=7)
    finally:
        _lib.call("avc_debug_xl_force_remote", 0)
    seen = (ctypes.c_uint * 2)()
    _lib.call("avc_debug_xl_census", seen)
    assert seen[1] >= 256 and seen[0] == 0, (seen[0], seen[1])  # every BPTT workgroup took the fallback
    for name, a, b in zip(["dx", "dW_ih", "dW_hh", "db_ih", "db_hh"], got, ref):
        assert torch.equal(a, b), name
