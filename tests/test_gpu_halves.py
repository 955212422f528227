"""Batch halves of the two-layer persistent recurrence (decoder.lstm2, lstm_persist_kernel NH = 2,
avc_lstm_persist_halves).

The workgroup walks its batch rows as two independent halves (step t of one half while the other
half's hand-off is in flight), on counters per (step, half).  LSTM batch rows never interact and
every row sees the same products in the same order, so the whole-Generator forward must be
bit-identical with and without halves -- eager, captured and replayed, at the batch sizes that
take each instance (RT = 2 x 2 tiles: B 33..64; 2 x 1: B 17..32), with the input-projection slot on
and off, and the give-up path must still leave NaN and raise.  The form is off by default (measured
slower); these tests switch it on."""
import ctypes

import pytest
import torch

from autovc_amd import _lib
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu


def _giveups():
    n = ctypes.c_long(0)
    _lib.call("avc_lstm_persist_status", ctypes.byref(n))
    return n.value


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


@pytest.mark.parametrize("B,T,inproj,training", [(64, 128, 1, True), (64, 128, 0, False), (48, 40, 1, True),
                                                 (33, 33, 1, True), (32, 96, 1, True), (17, 64, 0, True)])
def test_halves_are_bit_identical(cuda_device, B, T, inproj, training):
    ae = _model(cuda_device, training)
    x = torch.from_numpy(synthetic_mel(60 + B, B, T)).to(cuda_device)
    co = torch.from_numpy(synthetic_embedding(61, B)).to(cuda_device)
    ct = torch.from_numpy(synthetic_embedding(62, B)).to(cuda_device)
    before = _giveups()
    try:
        _lib.call("avc_lstm_persist_inproj", inproj)
        _lib.call("avc_lstm_persist_halves", 0)
        ref = _forwards(ae, x, co, ct)
        _lib.call("avc_lstm_persist_halves", 1)
        got = _forwards(ae, x, co, ct, reps=4)  # repeated launches: the epochs advance
    finally:
        _lib.call("avc_lstm_persist_halves", 0)
        _lib.call("avc_lstm_persist_inproj", 1)
    for run in got:
        for name, a, b in zip(("mel", "mel_post", "codes"), run, ref[0]):
            assert torch.equal(a, b), f"{name}: max|d| {(a - b).abs().max().item():.3e}"
    assert _giveups() == before


def test_halves_give_up_is_nan_and_next_call_raises(cuda_device):
    B, T = 64, 64
    ae = _model(cuda_device)
    x = torch.from_numpy(synthetic_mel(70, B, T)).to(cuda_device)
    c = torch.from_numpy(synthetic_embedding(71, B)).to(cuda_device)
    _lib.call("avc_graph_mode", 0)
    _lib.call("avc_lstm_persist_layers", 2)  # lstm2 is the forward's only persistent recurrence
    _lib.call("avc_lstm_persist_halves", 1)  # (off by default: measured slower)
    try:
        ref = _forwards(ae, x, c, c, reps=1)[0]
        before = _giveups()
        _lib.call("avc_debug_persist_inject", 1)
        with torch.no_grad():
            bad = [o.clone() for o in ae(x, c, c)]
        torch.cuda.synchronize()
        assert _giveups() > before
        assert torch.isnan(bad[1]).any(), "a forward whose recurrences gave up returned numbers"
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            ae.check_health()
        again = _forwards(ae, x, c, c, reps=1)[0]
    finally:
        _lib.call("avc_debug_persist_inject", 0)
        _lib.call("avc_lstm_persist_halves", 0)
        _lib.call("avc_lstm_persist_layers", 3)
        _lib.call("avc_graph_mode", 1)
    for a, b in zip(again, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,T", [(64, 128), (32, 96), (3, 40)])
def test_dead_h_stores_leave_outputs_unchanged(cuda_device, B, T):
    """avc_dead_h_stores: inside the whole-Generator forward the recurrences skip the fp32 h stores
    nothing reads (lstm2's layer 0; lstm1's and lstm2's last layer where the next contraction
    streams the split image).  The outputs must not change, eager and replayed."""
    ae = _model(cuda_device)
    x = torch.from_numpy(synthetic_mel(80 + B, B, T)).to(cuda_device)
    c = torch.from_numpy(synthetic_embedding(81, B)).to(cuda_device)
    try:
        _lib.call("avc_dead_h_stores", 0)
        ref = _forwards(ae, x, c, c)
        _lib.call("avc_dead_h_stores", 1)
        got = _forwards(ae, x, c, c)
    finally:
        _lib.call("avc_dead_h_stores", 1)
    for run in got:
        for a, b in zip(run, ref[0]):
            assert torch.equal(a, b)
