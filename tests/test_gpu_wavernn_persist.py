"""The persistent WaveRNN sample loop (avc_wavernn_persist(1)) against the per-step
graph-captured kernels (avc_wavernn_persist(0)).

The loop kernel runs every step of generate() in one launch with in-launch hand-offs, but each
of its phases forms its sums in the per-step kernels' order (the same lane split of every dot
product, the same fixed-order 64-lane reduction, the same gate and sampling expressions), so
samples, teacher-forced logits and the cross-faded waveform must agree bit for bit.  Cases:
one fold row (unbatched), 6 rows (one staging chunk) and 30 rows (two chunks), MOL and RAW, and
the reference's teacher-forced forward(x, mels).  A launch made to give up (test hook) must fail
the call with the device error and leave the context usable.
Reference: autovc/wavernn/model.py:180-329, distribution.py:87-123."""
import numpy as np
import pytest
import torch

from autovc_amd import _lib
from autovc_amd.weights import synthetic_mel, wavernn_state_dict
from autovc_amd.wavernn import WaveRNN
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu
DEFAULT = 1  # the library's default (avc_wavernn_persist)


@pytest.fixture(scope="module")
def sd():
    return wavernn_state_dict(0)


def make(dev, sd, mode="MOL"):
    net = WaveRNN(device=dev, mode=mode)
    net.load_state_dict({k: v for k, v in sd.items()})
    net.eval()
    return net


def _both(dev, fn):
    out = {}
    for mode in (0, 1):
        _lib.call("avc_wavernn_persist", mode)
        try:
            n0 = _lib.persist_launches(dev)
            res = fn()
            torch.cuda.synchronize()
            out[mode] = ([None if t is None else t.cpu().clone() for t in res], _lib.persist_launches(dev) - n0)
        finally:
            _lib.call("avc_wavernn_persist", DEFAULT)
    return out


@pytest.mark.parametrize("mode", ["MOL", "RAW"])
@pytest.mark.parametrize("T,batched,target,overlap", [(24, False, 0, 0), (24, True, 1000, 100), (120, True, 1000, 100)])
def test_loop_is_bit_identical(cuda_device, sd, mode, T, batched, target, overlap):
    if mode == "RAW":
        sd = dict(sd)
        g = torch.Generator().manual_seed(4)
        sd["fc3.weight"] = (torch.rand(18, 512, generator=g) - 0.5) * 0.2
        sd["fc3.bias"] = (torch.rand(18, generator=g) - 0.5) * 0.2
    net = make(cuda_device, sd, mode)
    mel = torch.from_numpy(synthetic_mel(21, 1, T))
    res = _both(cuda_device, lambda: net._run(mel, batched, target, overlap, 77))
    (s0, _, w0), n0 = res[0]
    (s1, _, w1), n1 = res[1]
    rows = s0.shape[0]
    assert n0 == 0, "the per-step path made a persistent launch"
    eligible = _lib.load().avc_wavernn_persist_eligible(rows, 512, 512)
    print(f"{mode} T={T}: {rows} fold rows x {s0.shape[1]} steps, persistent launches {n1}, eligible {eligible}")
    assert eligible == 1 and n1 == 1, "the persistent loop was not taken"
    assert torch.isfinite(s1).all()
    same = float((s0 == s1).double().mean())
    print(f"  samples bit-identical {100 * same:.3f} %, max |d| {float((s0 - s1).abs().max()):.2e}")
    assert torch.equal(s0, s1)
    assert torch.equal(w0, w1)


def test_teacher_forced_logits_are_bit_identical(cuda_device, sd):
    g = load_golden("wavernn_ref")
    net = make(cuda_device, sd)
    x, mels = torch.from_numpy(g["fwd_x"][:1]), torch.from_numpy(g["fwd_mels"][:1])
    res = _both(cuda_device, lambda: (net(x, mels),))
    (l0,), _ = res[0]
    (l1,), n1 = res[1]
    assert n1 == 1
    print(f"teacher-forced: {l0.shape[1]} steps, logits bit-identical {100 * float((l0 == l1).double().mean()):.3f} %")
    assert torch.equal(l0, l1)


def test_loop_give_up_is_reported_and_recovers(cuda_device, sd):
    net = make(cuda_device, sd)
    mel = torch.from_numpy(synthetic_mel(22, 1, 24))
    _lib.call("avc_wavernn_persist", 1)
    try:
        ref, _, _ = net._run(mel, True, 1000, 100, 5)
        torch.cuda.synchronize()
        _lib.call("avc_debug_wavernn_inject", 1)
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            net._run(mel, True, 1000, 100, 5)
        _lib.call("avc_debug_wavernn_inject", 0)
        again, _, _ = net._run(mel, True, 1000, 100, 5)  # fresh counter regions: same samples
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_debug_wavernn_inject", 0)
        _lib.call("avc_wavernn_persist", DEFAULT)
    assert torch.equal(ref.cpu(), again.cpu())


def test_eligibility_limits():
    # <= 96 fold rows, and fc1 + fc2 + sampling workgroups within the rnn_dims / 2 GRU workgroups
    assert _lib.load().avc_wavernn_persist_eligible(97, 512, 512) == 0
    assert _lib.load().avc_wavernn_persist_eligible(96, 512, 512) == 1
    assert _lib.load().avc_wavernn_persist_eligible(60, 256, 512) == 0


def test_tiled_input_projection_is_bit_identical(cuda_device, sd):
    """generate()'s per-position input projection pI (avc_wavernn_proj_tiled): the LDS-tiled kernel
    keeps every output's FMA chain order, so the whole generation is bit-identical."""
    net = make(cuda_device, sd)
    mel = torch.from_numpy(synthetic_mel(23, 1, 40))
    out = {}
    for mode in (0, 1):
        _lib.call("avc_wavernn_proj_tiled", mode)
        try:
            s, _, w = net._run(mel, True, 1000, 100, 9)
            torch.cuda.synchronize()
            out[mode] = (s.cpu(), w.cpu())
        finally:
            _lib.call("avc_wavernn_proj_tiled", 1)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    m, aux = net.upsample_features(mel)
    assert m.shape[0] == 40 * 275  # (the projection's rows: every position of the padded mel)
