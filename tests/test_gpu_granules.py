"""Granule hand-off of the one-layer persistent recurrence (lstm_persist.hip, gr_tag).

At H = 512 with one 16-row tile per batch group (decoder.lstm1 at C2 / C5 batch sizes) split h
goes from step to step as data-tagged 8-B granules instead of a counter hand-off.  The arithmetic
is the same, so outputs, saved gates / cell states (through the backward) and the give-up path
must match the counter form bit for bit."""
import ctypes

import pytest
import torch

from autovc_amd import _lib, ops

pytestmark = pytest.mark.gpu


def _giveups():
    n = ctypes.c_long(0)
    _lib.call("avc_lstm_persist_status", ctypes.byref(n))
    return n.value


def _layer(dev, T, B, din=320, H=512, seed=5):
    g = torch.Generator().manual_seed(seed)
    k = 1.0 / H ** 0.5
    ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev) for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    x = (torch.randn(T * B, din, generator=g) * 0.5).to(dev)
    dy = torch.randn(T * B, H, generator=g).to(dev)
    return ws, x, dy


def _run(ws, x, dy, T, B, save):
    ws = [w.clone().requires_grad_(save) for w in ws]
    x = x.clone().requires_grad_(save)
    y = ops.LSTMLayer.apply(x, *ws, T, B, save)
    if not save:
        return [y.detach()]
    y.backward(dy)
    return [y.detach(), x.grad] + [w.grad for w in ws]


@pytest.mark.parametrize("T,B,save", [(128, 64, False), (1024, 32, False), (40, 3, False), (64, 48, True),
                                      (33, 16, True)])
def test_granules_match_counter_form(cuda_device, T, B, save):
    ws, x, dy = _layer(cuda_device, T, B)
    before = _giveups()
    _lib.call("avc_lstm_persist_granules", 0)  # (the library default since round 4)
    ref = _run(ws, x, dy, T, B, save)
    _lib.call("avc_lstm_persist_granules", 1)
    try:
        for _ in range(3):  # repeated launches on one counter region: epochs and ring tags advance
            got = _run(ws, x, dy, T, B, save)
            for a, b in zip(got, ref):
                assert torch.equal(a, b)
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_lstm_persist_granules", 0)
    assert _giveups() == before


def test_granule_give_up_is_nan_and_next_call_raises(cuda_device):
    T, B = 64, 32
    ws, x, dy = _layer(cuda_device, T, B)
    _lib.call("avc_lstm_persist_granules", 1)
    try:
        ref = _run(ws, x, dy, T, B, False)[0]
        torch.cuda.synchronize()
        before = _giveups()
        _lib.call("avc_debug_persist_inject", 1)
        bad = ops.LSTMLayer.apply(x, *ws, T, B, False)
        torch.cuda.synchronize()
        assert _giveups() > before
        assert torch.isnan(bad).any(), "timed-out launch returned numbers"
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            ops.LSTMLayer.apply(x, *ws, T, B, False)
        assert torch.equal(_run(ws, x, dy, T, B, False)[0], ref)
    finally:
        _lib.call("avc_debug_persist_inject", 0)
        _lib.call("avc_lstm_persist_granules", 0)
