"""XCD-local groups in the one-layer persistent recurrence (avc_lstm_persist_xcd, PersistArgs::xl,
round 5).  Each batch group's workgroups are dealt to one XCD; a run-time check confirms it and the
group then hands h over with plain stores that stay in that XCD's L2, read there by its consumers'
sc1 loads.  The products, their order and the epilogue are unchanged, so outputs (and, through
the saved activations, every gradient) must equal the write-through form bit for bit -- eager,
captured and replayed, over repeated launches on one region, at the C2 / C5 batches and ragged
ones.  Reference layer: autovc/auto_encoder/decoder.py:50,69 (lstm1)."""
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


def _forwards(ae, x, co, ct, reps):
    outs = []
    with torch.no_grad():
        for _ in range(reps):  # eager, capture + replay, replays
            outs.append([o.clone() for o in ae(x, co, ct)])
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("B,T,training", [(64, 128, True), (32, 1024, True), (64, 128, False), (17, 96, True),
                                          (3, 200, True), (1, 300, True), (48, 64, True)])
def test_xcd_local_forward_is_bit_identical(cuda_device, B, T, training):
    ae = _model(cuda_device, training)
    x = torch.from_numpy(synthetic_mel(200 + B, B, T)).to(cuda_device)
    co = torch.from_numpy(synthetic_embedding(201, B)).to(cuda_device)
    ct = torch.from_numpy(synthetic_embedding(202, B)).to(cuda_device)
    before = _giveups()
    try:
        _lib.call("avc_lstm_persist_xcd", 0)
        ref = _forwards(ae, x, co, ct, 2)
        _lib.call("avc_lstm_persist_xcd", 1)
        got = _forwards(ae, x, co, ct, 6)
    finally:
        _lib.call("avc_lstm_persist_xcd", 0)  # (the default)
    for run in got:
        for name, a, b in zip(("mel", "mel_post", "codes"), run, ref[0]):
            assert torch.equal(a, b), f"{name}: max|d| {(a - b).abs().max().item():.3e}"
    assert _giveups() == before
    seen = (ctypes.c_uint * 2)()
    _lib.call("avc_debug_xl_census", seen)
    print(f"B={B} T={T}: recurrent workgroups local {seen[0]}, not local {seen[1]}")


def test_xcd_local_training_step_is_bit_identical(cuda_device):
    B, T = 64, 128
    X = torch.from_numpy(synthetic_mel(203, B, T)).to(cuda_device)
    c = torch.from_numpy(synthetic_embedding(204, B)).to(cuda_device)
    res = []
    for on in (0, 1, 1):
        ae = _model(cuda_device)
        ae.configure_optimizer()
        _lib.call("avc_lstm_persist_xcd", on)
        try:
            for _ in range(2):
                loss, norm = ae.train_step(X, c)
            torch.cuda.synchronize()
        finally:
            _lib.call("avc_lstm_persist_xcd", 0)  # (the default)
        res.append((loss.item(), norm.item(), ae._flat_param.detach().clone()))
    for r in res[1:]:
        assert r[0] == res[0][0] and r[1] == res[0][1]
        assert torch.equal(r[2], res[0][2])


@pytest.mark.parametrize("B,T", [(64, 128), (32, 300)])
def test_xcd_local_fallback_is_bit_identical(cuda_device, B, T):
    """XL groups found not local (forced: avc_debug_xl_force_remote) keep the write-through stores
    and counters on the linear grid -- the same bits as the round-4 grid."""
    ae = _model(cuda_device, True)
    x = torch.from_numpy(synthetic_mel(300 + B, B, T)).to(cuda_device)
    co = torch.from_numpy(synthetic_embedding(301, B)).to(cuda_device)
    ct = torch.from_numpy(synthetic_embedding(302, B)).to(cuda_device)
    ref = _forwards(ae, x, co, ct, 2)
    _lib.call("avc_debug_xl_census", (ctypes.c_uint * 2)())  # (clear)
    try:
        _lib.call("avc_lstm_persist_xcd", 1)
        _lib.call("avc_debug_xl_force_remote", 1)
        got = _forwards(ae, x, co, ct, 4)
    finally:
        _lib.call("avc_debug_xl_force_remote", 0)
        _lib.call("avc_lstm_persist_xcd", 0)  # (the default)
    seen = (ctypes.c_uint * 2)()
    _lib.call("avc_debug_xl_census", seen)
    assert seen[0] == 0 and seen[1] > 0, (seen[0], seen[1])
    for run in got:
        for a, b in zip(run, ref[0]):
            assert torch.equal(a, b)
