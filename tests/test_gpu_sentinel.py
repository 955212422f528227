"""Sentinel hand-off of split h in the persistent recurrences (lstm_persist_kernel SN,
avc_lstm_persist_sentinel).

The split-h buffers live in the launch's region, two sets chosen by the launch epoch's parity, and
every byte of the set a launch uses is 0xFF until its producer writes it.  Consumers re-load an h
chunk until none of its dwords is the sentinel, instead of waiting on arrival counters; each
producer resets its bytes of the other set for the next launch.  The products and their order are
unchanged, so outputs (and, with saved activations, every gradient of the backward) must equal the
counter form bit for bit -- eager, captured and replayed, over repeated launches (the sets
alternate), for the one-layer form (decoder.lstm1, bit 1) and the two-layer form (decoder.lstm2,
bit 0) -- and a launch that gives up must still leave NaN and make the next call raise.
Reference layers: autovc/auto_encoder/decoder.py:50,53,69,74."""
import ctypes

import pytest
import torch

from autovc_amd import _lib, ops
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu
DEFAULT = 0  # the library's default (avc_lstm_persist_sentinel)


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
                                      (33, 16, True), (20, 256, True)])
def test_one_layer_sentinel_matches_counter_form(cuda_device, T, B, save):
    ws, x, dy = _layer(cuda_device, T, B)
    before = _giveups()
    _lib.call("avc_lstm_persist_sentinel", 0)
    ref = _run(ws, x, dy, T, B, save)
    _lib.call("avc_lstm_persist_sentinel", 2)
    try:
        for _ in range(3):  # repeated launches on one region: the sets alternate
            got = _run(ws, x, dy, T, B, save)
            for a, b in zip(got, ref):
                assert torch.equal(a, b), f"max|d| {(a - b).abs().max().item():.3e}"
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_lstm_persist_sentinel", DEFAULT)
    assert _giveups() == before


def _model(dev, training=True):
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    return ae.to(dev).train(training)


def _forwards(ae, x, co, ct, reps=3):
    outs = []
    with torch.no_grad():
        for _ in range(reps):  # eager, capture + replay, replay
            outs.append([o.clone() for o in ae(x, co, ct)])
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("B,T,inproj,training", [(64, 128, 1, True), (64, 128, 0, False), (32, 1000, 1, True),
                                                 (48, 40, 1, True), (17, 64, 0, True), (3, 96, 1, True),
                                                 (1, 300, 1, True)])
def test_whole_forward_sentinel_is_bit_identical(cuda_device, B, T, inproj, training):
    ae = _model(cuda_device, training)
    x = torch.from_numpy(synthetic_mel(90 + B, B, T)).to(cuda_device)
    co = torch.from_numpy(synthetic_embedding(91, B)).to(cuda_device)
    ct = torch.from_numpy(synthetic_embedding(92, B)).to(cuda_device)
    before = _giveups()
    try:
        _lib.call("avc_lstm_persist_inproj", inproj)
        _lib.call("avc_lstm_persist_sentinel", 0)
        ref = _forwards(ae, x, co, ct)
        _lib.call("avc_lstm_persist_sentinel", 3)
        got = _forwards(ae, x, co, ct, reps=5)  # the sets alternate launch by launch
    finally:
        _lib.call("avc_lstm_persist_sentinel", DEFAULT)
        _lib.call("avc_lstm_persist_inproj", 1)
    for run in got:
        for name, a, b in zip(("mel", "mel_post", "codes"), run, ref[0]):
            assert torch.equal(a, b), f"{name}: max|d| {(a - b).abs().max().item():.3e}"
    assert _giveups() == before


def test_training_step_sentinel_is_bit_identical(cuda_device):
    """One C3-shaped training step (B = 256 rows: the one-layer form in 64-row groups, the
    two-layer form's saved gates and cell states feeding the persistent BPTT) with and without the
    sentinel hand-off: same loss, gradient norm and parameters."""
    B, T = 256, 64
    X = torch.from_numpy(synthetic_mel(93, B, T)).to(cuda_device)
    c = torch.from_numpy(synthetic_embedding(94, B)).to(cuda_device)
    res = []
    for mask in (0, 3):
        ae = _model(cuda_device)
        ae.configure_optimizer()
        _lib.call("avc_lstm_persist_sentinel", mask)
        try:
            loss, norm = ae.train_step(X, c)
            torch.cuda.synchronize()
        finally:
            _lib.call("avc_lstm_persist_sentinel", DEFAULT)
        res.append((loss.item(), norm.item(), ae._flat_param.detach().clone()))
    assert res[0][0] == res[1][0] and res[0][1] == res[1][1]
    assert torch.equal(res[0][2], res[1][2])


@pytest.mark.parametrize("layers", [1, 2])
def test_sentinel_give_up_is_nan_and_next_call_raises(cuda_device, layers):
    B, T = 64, 64
    ae = _model(cuda_device)
    x = torch.from_numpy(synthetic_mel(95, B, T)).to(cuda_device)
    c = torch.from_numpy(synthetic_embedding(96, B)).to(cuda_device)
    _lib.call("avc_graph_mode", 0)
    _lib.call("avc_lstm_persist_layers", layers)  # the forward's only persistent recurrence
    _lib.call("avc_lstm_persist_sentinel", 3)
    try:
        ref = _forwards(ae, x, c, c, reps=1)[0]
        before = _giveups()
        _lib.call("avc_debug_persist_inject", 1)
        with torch.no_grad():
            bad = [o.clone() for o in ae(x, c, c)]
        torch.cuda.synchronize()
        assert _giveups() > before
        assert torch.isnan(bad[1]).any(), "a forward whose recurrence gave up returned numbers"
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            ae.check_health()
        again = _forwards(ae, x, c, c, reps=2)  # fresh regions (sentinel-filled), then the other set
    finally:
        _lib.call("avc_debug_persist_inject", 0)
        _lib.call("avc_lstm_persist_sentinel", DEFAULT)
        _lib.call("avc_lstm_persist_layers", 3)
        _lib.call("avc_graph_mode", 1)
    for run in again:
        for a, b in zip(run, ref):
            assert torch.equal(a, b)


@pytest.mark.parametrize("B,T,sn", [(64, 128, 0), (32, 200, 0), (3, 50, 0), (64, 64, 3), (256, 32, 0)])
def test_16_byte_hand_off_stores_are_bit_identical(cuda_device, B, T, sn):
    """avc_lstm_persist_st16 (round 5): the split-h hand-off as one 16-B write-through piece per
    pair lead (halves exchanged by a lane shuffle) instead of two 8-B stores; the same bytes land."""
    ae = _model(cuda_device)
    x = torch.from_numpy(synthetic_mel(97 + B, B, T)).to(cuda_device)
    c = torch.from_numpy(synthetic_embedding(98, B)).to(cuda_device)
    try:
        _lib.call("avc_lstm_persist_sentinel", sn)
        _lib.call("avc_lstm_persist_st16", 0)
        ref = _forwards(ae, x, c, c)
        _lib.call("avc_lstm_persist_st16", 1)
        got = _forwards(ae, x, c, c)
    finally:
        _lib.call("avc_lstm_persist_st16", 1)
        _lib.call("avc_lstm_persist_sentinel", DEFAULT)
    for run in got:
        for a, b in zip(run, ref[0]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("B,T,training", [(64, 128, True), (32, 1000, False), (48, 40, True), (17, 64, True),
                                          (256, 32, True)])
def test_chunk_waits_are_bit_identical(cuda_device, B, T, training):
    """avc_lstm_persist_chunkwait (round 5): the two-layer form's waves wait per 32-deep h chunk
    (two producing workgroups) instead of per K quarter; the products and their order are unchanged."""
    ae = _model(cuda_device, training)
    x = torch.from_numpy(synthetic_mel(99 + B, B, T)).to(cuda_device)
    c = torch.from_numpy(synthetic_embedding(100, B)).to(cuda_device)
    before = _giveups()
    try:
        _lib.call("avc_lstm_persist_chunkwait", 0)
        ref = _forwards(ae, x, c, c)
        _lib.call("avc_lstm_persist_chunkwait", 1)
        got = _forwards(ae, x, c, c)
    finally:
        _lib.call("avc_lstm_persist_chunkwait", 0)
    for run in got:
        for a, b in zip(run, ref[0]):
            assert torch.equal(a, b), f"max|d| {(a - b).abs().max().item():.3e}"
    assert _giveups() == before


def test_chunk_wait_give_up_is_nan_and_next_call_raises(cuda_device):
    B, T = 64, 64
    ae = _model(cuda_device)
    x = torch.from_numpy(synthetic_mel(101, B, T)).to(cuda_device)
    c = torch.from_numpy(synthetic_embedding(102, B)).to(cuda_device)
    _lib.call("avc_graph_mode", 0)
    _lib.call("avc_lstm_persist_layers", 2)
    _lib.call("avc_lstm_persist_chunkwait", 1)
    try:
        ref = _forwards(ae, x, c, c, reps=1)[0]
        before = _giveups()
        _lib.call("avc_debug_persist_inject", 1)
        with torch.no_grad():
            bad = [o.clone() for o in ae(x, c, c)]
        torch.cuda.synchronize()
        assert _giveups() > before
        assert torch.isnan(bad[1]).any(), "a forward whose recurrence gave up returned numbers"
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            ae.check_health()
        again = _forwards(ae, x, c, c, reps=2)
    finally:
        _lib.call("avc_debug_persist_inject", 0)
        _lib.call("avc_lstm_persist_chunkwait", 0)
        _lib.call("avc_lstm_persist_layers", 3)
        _lib.call("avc_graph_mode", 1)
    for run in again:
        for a, b in zip(run, ref):
            assert torch.equal(a, b)
