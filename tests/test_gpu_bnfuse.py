"""BatchNorm fused into the convolution's GEMM epilogue (gemm.h BnFuse, avc_bn_fuse).

Reference composition: ConvNorm -> BatchNorm1d -> relu / tanh / identity (encoder.py:69-70,
decoder.py:69-70, postnet.py:54-61), with model.py:131-132's residual on postnet's last layer.
The fused form keeps y = conv(x) in registers, forms mean / invstd in every workgroup from the
column partials behind a column-tile barrier (train mode) or from the running statistics (eval
mode), and writes the normalised output and its split image.  Every value is formed by the same
expressions in the same order as the unfused chain (GEMM -> bn_finalize -> bn_apply), so outputs,
y_pre, mean / invstd and the running statistics must be bit-identical -- at one co-resident wave of
workgroups (C2's 256) and at small grids, in both BN modes, across repeated launches (epochs) and
HIP-graph replays of the whole-Generator forward."""
import ctypes
import time

import pytest
import torch

from autovc_amd import _lib
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu

RELU, TANH, NONE = 1, 2, 0


def _fuse(on):
    _lib.call("avc_bn_fuse", int(on))


@pytest.fixture(autouse=True)
def _restore_default():
    yield
    _fuse(1)


def _conv_inputs(dev, T, B, cin, cout, residual, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(T * B, cin, generator=g)).to(dev)
    W = ((torch.rand(cout, cin, 5, generator=g) - 0.5) * 0.2).to(dev)
    bias = ((torch.rand(cout, generator=g) - 0.5) * 0.1).to(dev)
    gamma = (torch.rand(cout, generator=g) + 0.5).to(dev)
    beta = ((torch.rand(cout, generator=g) - 0.5) * 0.2).to(dev)
    rm = ((torch.rand(cout, generator=g) - 0.5) * 0.1).to(dev)
    rv = (torch.rand(cout, generator=g) + 0.5).to(dev)
    res = torch.randn(T * B, cout, generator=g).to(dev) if residual else None
    y_pre = torch.full((T * B, cout), float("nan"), device=dev)
    out = torch.full((T * B, cout), float("nan"), device=dev)
    mean = torch.zeros(cout, device=dev)
    invstd = torch.zeros(cout, device=dev)
    return x, W, bias, gamma, beta, rm, rv, res, y_pre, out, mean, invstd


def _conv_call(dev, T, B, cin, cout, act, training, t):
    x, W, bias, gamma, beta, rm, rv, res, y_pre, out, mean, invstd = t
    _lib.call("avc_conv_bn_act_forward", _lib.context(dev), T, B, cin, cout, _lib.ptr(x), _lib.ptr(W),
              _lib.ptr(bias), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(rm), _lib.ptr(rv), int(training),
              ctypes.c_float(0.1), ctypes.c_float(1e-5), act, _lib.ptr(res), _lib.ptr(y_pre), _lib.ptr(out),
              _lib.ptr(mean), _lib.ptr(invstd), _lib.stream(dev))


def _conv(dev, T, B, cin, cout, act, training, residual, seed, reps=1):
    t = _conv_inputs(dev, T, B, cin, cout, residual, seed)
    outs = []
    for _ in range(reps):
        _conv_call(dev, T, B, cin, cout, act, training, t)
        torch.cuda.synchronize()
        x, W, bias, gamma, beta, rm, rv, res, y_pre, out, mean, invstd = t
        outs.append([v.clone() for v in (out, y_pre, mean, invstd, rm, rv)])
    return outs


@pytest.mark.parametrize("T,B,cin,cout,act,residual", [
    (128, 64, 512, 512, RELU, False),   # C2 conv: 64 x 4 tiles of 128 x 128, one per CU
    (128, 64, 336, 512, RELU, False),   # encoder's first conv (cin = 80 + 256)
    (128, 64, 512, 80, NONE, True),     # postnet's last conv + residual: 64 x 64 tiles
    (128, 2, 512, 512, TANH, False),    # a small grid (8 workgroups)
    (96, 3, 80, 512, TANH, False),      # ragged rows: M = 288
])
@pytest.mark.parametrize("training", [True, False])
def test_fused_conv_bn_is_bit_identical(cuda_device, T, B, cin, cout, act, residual, training):
    _fuse(0)
    ref = _conv(cuda_device, T, B, cin, cout, act, training, residual, seed=5, reps=2)
    _fuse(1)
    got = _conv(cuda_device, T, B, cin, cout, act, training, residual, seed=5, reps=2)
    names = ["out", "y_pre", "mean", "invstd", "running_mean", "running_var"]
    bad = []
    for rep in range(2):  # the second launch runs at the next epoch of the same counters
        for n, a, b in zip(names, got[rep], ref[rep]):
            if not torch.equal(a, b):
                d = (a.double() - b.double()).abs().nan_to_num(9.0)
                bad.append((rep, n, float(d.max()), int((d > 0).sum()), a.numel()))
    assert not bad, bad
    assert torch.isfinite(got[1][0]).all()


@pytest.mark.parametrize("training", [True, False])
def test_fused_conv_bn_multi_wave_is_bit_identical(cuda_device, training):
    """avc_bn_fuse(2): the fused form on a grid of several waves (C3's conv, B = 256: 1024
    workgroups, 4 column groups of 256 that pass their barriers one after another) gives the
    unfused chain's bits, across two launches (epochs)."""
    shape = (128, 256, 512, 512, RELU, False)
    try:
        _fuse(0)
        ref = _conv(cuda_device, *shape[:5], training, shape[5], seed=6, reps=2)
        _fuse(2)
        launches = _lib.persist_launches(cuda_device)
        got = _conv(cuda_device, *shape[:5], training, shape[5], seed=6, reps=2)
        if training:
            assert _lib.persist_launches(cuda_device) - launches == 2  # the fused form ran
    finally:
        _fuse(1)
    for rep in range(2):
        for a, b in zip(got[rep], ref[rep]):
            assert torch.equal(a, b)


def test_fused_conv_bn_is_taken_at_c2():
    """The C2 conv products take the fused form (one co-resident wave: 256 tiles of 128 x 128)."""
    lib = _lib.load()
    assert lib.avc_conv_frag_chain_ok(128, 64, 512, 512) == 1


def _generator(dev, training, reps, B=64, T=128):
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    ae.to(dev)
    ae.train(training)
    x = torch.from_numpy(synthetic_mel(11, B, T)).to(dev)
    c = torch.from_numpy(synthetic_embedding(12, B)).to(dev)
    outs = []
    with torch.no_grad():
        for _ in range(reps):  # eager, then captured, then replayed
            mel, post, codes = ae(x, c, c)
            torch.cuda.synchronize()
            bufs = [b.detach().clone() for n, b in ae.named_buffers() if "running" in n]
            outs.append([mel.clone(), post.clone(), codes.clone()] + bufs)
    ae.check_health()
    return outs


@pytest.mark.parametrize("training", [True, False])
def test_whole_generator_fused_bn_is_bit_identical(cuda_device, training):
    _fuse(0)
    ref = _generator(cuda_device, training, reps=4)
    _fuse(1)
    got = _generator(cuda_device, training, reps=4)
    for rep in range(4):
        for i, (a, b) in enumerate(zip(got[rep], ref[rep])):
            assert torch.equal(a, b), (rep, i, float((a.double() - b.double()).abs().max()))


@pytest.mark.parametrize("training", [True, False])
def test_fused_bn_dispatch_band_is_bit_identical(cuda_device, training):
    """avc_bn_fuse_band (round 5): XCD-contiguous row bands per column group vs round 4's order.
    Only which workgroup computes which tile changes, so the whole Generator forward is identical."""
    _fuse(1)
    try:
        _lib.call("avc_bn_fuse_band", 0)
        ref = _generator(cuda_device, training, reps=3)
        _lib.call("avc_bn_fuse_band", 1)
        got = _generator(cuda_device, training, reps=3)
    finally:
        _lib.call("avc_bn_fuse_band", 1)
    for rep in range(3):
        for i, (a, b) in enumerate(zip(got[rep], ref[rep])):
            assert torch.equal(a, b), (rep, i, float((a.double() - b.double()).abs().max()))


def _set_handover(on):
    _lib.call("avc_split_handover", int(on))


@pytest.mark.parametrize("training", [True, False])
def test_split_handovers_are_bit_identical(cuda_device, training):
    """The encoder's last conv -> BiLSTM projection, lstm1 -> first decoder conv and lstm2 -> Linear
    hand-overs as split images written by the producers (avc_split_handover) give the bits of the
    fp32 hand-over + split pass, at C2 (B = 64: every hand-over active)."""
    try:
        _set_handover(0)
        ref = _generator(cuda_device, training, reps=3)
        _set_handover(1)
        got = _generator(cuda_device, training, reps=3)
    finally:
        _set_handover(1)
    for rep in range(3):
        for i, (a, b) in enumerate(zip(got[rep], ref[rep])):
            assert torch.equal(a, b), (rep, i, float((a.double() - b.double()).abs().max()))


# The two fused instances at C2 shapes: 128 x 128 tiles (tilesM = 64 row tiles per column tile,
# one workgroup per CU) and postnet's last conv on 64 x 64 tiles (tilesM = 128, two per CU).  Either
# way one barrier group needs 64 CUs: 8 on each XCD, since a group is a contiguous dispatch range
# dealt round-robin over the 8 XCDs.
HELD_SHAPES = [(128, 64, 512, 512, RELU, False), (128, 64, 512, 80, NONE, True)]


def _hold_cus(dev, n_hold, stream):
    """Start avc_debug_hog with n_hold workgroups of 160 KB LDS (one per CU) for 0.6 s on `stream`
    and wait until all of them run; returns how many it holds on each XCD."""
    _lib.call("avc_debug_hog", _lib.context(dev), n_hold, 160 * 1024, 600_000, stream.cuda_stream)
    n, t0 = ctypes.c_int(0), time.time()
    while n.value < n_hold and time.time() - t0 < 20:
        _lib.call("avc_debug_hog_resident", _lib.context(dev), ctypes.byref(n))
        time.sleep(0.001)
    assert n.value == n_hold
    per = (ctypes.c_int * 8)()
    _lib.call("avc_debug_hog_xcds", _lib.context(dev), per)
    return list(per)


def _fused_conv_beside_hog(dev, shape, n_hold, seed):
    """One train-mode fused conv dispatched while n_hold CUs are held by a kernel on another
    stream, with the barrier's bounded wait cut to 2^13 polls.  Returns (reference outputs, outputs,
    gave_up, held per XCD)."""
    T, B, cin, cout, act, residual = shape
    ref = _conv(dev, T, B, cin, cout, act, True, residual, seed=seed)[0]
    t = _conv_inputs(dev, T, B, cin, cout, residual, seed=seed)  # everything ready before the CUs are held
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    _lib.call("avc_debug_persist_spin_limit", 1 << 13)
    try:
        side.wait_stream(torch.cuda.current_stream(dev))
        per = _hold_cus(dev, n_hold, side)
        launches = _lib.persist_launches(dev)
        _conv_call(dev, T, B, cin, cout, act, True, t)  # dispatches while the CUs are held
        torch.cuda.synchronize()
        assert _lib.persist_launches(dev) - launches == 1  # the fused, co-resident form ran
    finally:
        _lib.call("avc_debug_persist_spin_limit", 0)
    got = [v.clone() for v in (t[9], t[8], t[10], t[11], t[5], t[6])]
    try:
        _lib.call("avc_persist_check", _lib.context(dev), _lib.stream(dev), None)
        gave_up = False
    except RuntimeError as e:
        assert "abandoned a bounded wait" in str(e)
        gave_up = True
    return ref, got, gave_up, per


@pytest.mark.parametrize("shape", HELD_SHAPES, ids=["128x128", "64x64"])
def test_fused_conv_bn_needs_only_one_column_group(cuda_device, shape):
    """Positive control of the co-residency invariant: with every CU but 8 per XCD
    held, the 256-workgroup grid is far from co-resident, but each column tile's group (a
    contiguous dispatch range, 8 per XCD) is; the groups pass their barriers one after another and
    the result equals the unfused chain bit for bit."""
    cus = torch.cuda.get_device_properties(cuda_device).multi_processor_count
    if cus % 8:
        pytest.skip(f"{cus} CUs: not 8 equal XCDs")
    ref, got, gave_up, per = _fused_conv_beside_hog(cuda_device, shape, cus - 64, seed=9)
    free = [cus // 8 - p for p in per]
    print("held per XCD", per, "free", free)
    if min(free) < 8:
        pytest.skip(f"the hog was not dealt evenly over the XCDs ({per}): no control")
    assert not gave_up, f"a group of 8 per XCD had 8 free CUs per XCD and still gave up ({per})"
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", HELD_SHAPES, ids=["128x128", "64x64"])
def test_fused_conv_bn_gives_up_beside_held_cus(cuda_device, shape):
    """Negative control under real contention: hold all but 56 CUs (at least one XCD keeps at
    most 7 free, fewer than the 8 one column group places there; 56 free in total is fewer than
    the group's 64 on any placement).  The first group can never be resident at once, so its
    barrier must give up within the bounded wait: NaN outputs, a raise on the next check, and after
    that reset the same call gives the reference bits again."""
    cus = torch.cuda.get_device_properties(cuda_device).multi_processor_count
    ref, got, gave_up, per = _fused_conv_beside_hog(cuda_device, shape, cus - 56, seed=10)
    print("held per XCD", per, "free", [cus // 8 - p for p in per])
    assert gave_up, f"the barrier passed with only 56 CUs free ({per})"
    assert torch.isnan(got[0]).any(), "a fused conv that gave up returned only numbers"
    T, B, cin, cout, act, residual = shape
    again = _conv(cuda_device, T, B, cin, cout, act, True, residual, seed=10)[0]
    for a, b in zip(again, ref):
        assert torch.equal(a, b)


def test_fused_conv_bn_give_up_is_nan_and_reported(cuda_device):
    """The barrier's bounded wait, forced (avc_debug_bnf_inject): the launch gives up instead of
    waiting, its output carries NaN, the next check on the context raises, and after that reset
    the same call gives the reference bits again (a fresh counter region)."""
    dev = cuda_device
    ref = _conv(dev, 128, 64, 512, 512, RELU, True, False, seed=13)[0]
    _lib.call("avc_debug_bnf_inject", 1)
    try:
        bad = _conv(dev, 128, 64, 512, 512, RELU, True, False, seed=13)[0]
    finally:
        _lib.call("avc_debug_bnf_inject", 0)
    assert torch.isnan(bad[0]).any(), "a fused conv that gave up returned only numbers"
    with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
        _lib.call("avc_persist_check", _lib.context(dev), _lib.stream(dev), None)
    again = _conv(dev, 128, 64, 512, 512, RELU, True, False, seed=13)[0]
    for a, b in zip(again, ref):
        assert torch.equal(a, b)
