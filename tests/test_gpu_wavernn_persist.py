"""The persistent WaveRNN sample loop (avc_wavernn_persist(1)) against the per-step
graph-captured kernels (avc_wavernn_persist(0)).

The loop kernel runs every step of generate() in one launch with in-launch hand-offs, but each
of its phases forms its sums in the per-step kernels' order (the same lane split of every dot
product, the same fixed-order 64-lane reduction, the same gate and sampling expressions), so
samples, teacher-forced logits and the cross-faded waveform must agree bit for bit.  Cases:
one fold row (unbatched), 6 rows (one staging chunk) and 30 rows (two chunks), MOL and RAW, and
the reference's teacher-forced forward(x, mels), and 73-96 rows (all four staging chunks).  A launch
that gives up (test hook, or CUs held by another kernel) is re-run per step by the same call.
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


def test_loop_give_up_falls_back_to_the_per_step_path(cuda_device, sd):
    """A loop launch that gives up (test hook) is re-run by the same call on the per-step graph
    path: the call succeeds with the same samples, and the next call takes the loop again."""
    net = make(cuda_device, sd)
    mel = torch.from_numpy(synthetic_mel(22, 1, 24))
    lib = _lib.load()
    _lib.call("avc_wavernn_persist", 1)
    try:
        ref, _, wref = net._run(mel, True, 1000, 100, 5)
        torch.cuda.synchronize()
        f0 = lib.avc_wavernn_fallbacks()
        _lib.call("avc_debug_wavernn_inject", 1)
        got, _, wgot = net._run(mel, True, 1000, 100, 5)
        torch.cuda.synchronize()
        _lib.call("avc_debug_wavernn_inject", 0)
        assert lib.avc_wavernn_fallbacks() == f0 + 1, "the injected give-up was not re-run per step"
        n0 = _lib.persist_launches(cuda_device)
        again, _, _ = net._run(mel, True, 1000, 100, 5)  # fresh counter regions: the loop again
        torch.cuda.synchronize()
        assert _lib.persist_launches(cuda_device) - n0 == 1
        assert lib.avc_wavernn_fallbacks() == f0 + 1
    finally:
        _lib.call("avc_debug_wavernn_inject", 0)
        _lib.call("avc_wavernn_persist", DEFAULT)
    assert torch.equal(ref.cpu(), got.cpu()) and torch.equal(wref.cpu(), wgot.cpu())
    assert torch.equal(ref.cpu(), again.cpu())


def test_loop_beside_held_cus_still_generates(cuda_device, sd):
    """the loop holds one workgroup on every CU it uses for the whole call.  With 192
    CUs held by another kernel (a 160 KB-LDS hog on a side stream) its 256-workgroup grid cannot
    be resident; the launch gives up within its (shortened) bounded wait and the call completes on
    the per-step path with the same samples."""
    import ctypes
    import time
    net = make(cuda_device, sd)
    mel = torch.from_numpy(synthetic_mel(24, 1, 24))
    lib = _lib.load()
    ref, _, _ = net._run(mel, True, 1000, 100, 6)
    torch.cuda.synchronize()
    cus = torch.cuda.get_device_properties(cuda_device).multi_processor_count
    n_hold = cus - 64
    side = torch.cuda.Stream(device=cuda_device)
    f0 = lib.avc_wavernn_fallbacks()
    _lib.call("avc_debug_persist_spin_limit", 1 << 13)
    try:
        side.wait_stream(torch.cuda.current_stream(cuda_device))
        _lib.call("avc_debug_hog", _lib.context(cuda_device), n_hold, 160 * 1024, 600_000, side.cuda_stream)
        n, t0 = ctypes.c_int(0), time.time()
        while n.value < n_hold and time.time() - t0 < 20:
            _lib.call("avc_debug_hog_resident", _lib.context(cuda_device), ctypes.byref(n))
            time.sleep(0.001)
        assert n.value == n_hold
        got, _, _ = net._run(mel, True, 1000, 100, 6)
        torch.cuda.synchronize()
    finally:
        _lib.call("avc_debug_persist_spin_limit", 0)
    print(f"held {n_hold} CUs; fallbacks {lib.avc_wavernn_fallbacks() - f0}")
    assert lib.avc_wavernn_fallbacks() == f0 + 1, "the loop did not give up beside 192 held CUs"
    assert torch.equal(ref.cpu(), got.cpu())
    _lib.call("avc_persist_check", _lib.context(cuda_device), _lib.stream(cuda_device), None)


@pytest.mark.parametrize("T", [300])
def test_loop_four_staging_chunks(cuda_device, sd, T):
    """a batched call with 73-96 fold rows fills all four staging chunks of the loop
    (kWrMaxChunks = 4, 24 rows each): bit-identical to the per-step path."""
    net = make(cuda_device, sd)
    mel = torch.from_numpy(synthetic_mel(25, 1, T))
    res = _both(cuda_device, lambda: net._run(mel, True, 1000, 100, 31))
    (s0, _, w0), _ = res[0]
    (s1, _, w1), n1 = res[1]
    rows = s0.shape[0]
    print(f"{rows} fold rows x {s0.shape[1]} steps")
    assert 73 <= rows <= 96 and n1 == 1
    assert torch.equal(s0, s1) and torch.equal(w0, w1)


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
