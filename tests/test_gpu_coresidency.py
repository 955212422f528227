"""Co-residency of the persistent launches beside a collective that holds CUs (BASELINE
config 4's per-rank plan; reference training step autovc/auto_encoder/model.py:312-318).

The persistent BPTT (lstm_persist.hip: bptt_persist_kernel) needs all 256 CUs at once.  In data-
parallel training an RCCL kernel waiting for a lagging peer can hold CUs; if it does while the
BPTT dispatches, the BPTT's resident workgroups spin until their bounded wait gives up.  The rule
(dp.GradBuckets): no collective is in flight while a persistent launch dispatches.

The collective here is a stand-in driven through the real bucketed exchange (AutoEncoder.grad_comm
-> dp.GradBuckets): each bucket's "all-reduce" launches a kernel on a side stream that holds 192
whole CUs (160 KB of LDS each) for far longer than the spin limit, and the host waits until it is
resident before going on -- the worst case of a peer that is late.  The spin limit is cut to 2^13
polls (about a millisecond) so a give-up shows within the test.  (At B = 256 the BPTT's 256
workgroups form two independent 128-workgroup row groups, so with up to 128 CUs held one group
finishes, leaves, and the other one gets its CUs: the launch is late but completes.  Holding 192
CUs leaves neither group whole.)
  * with the rule off the BPTT dispatches beside the held CUs and gives up (the hazard is real);
  * with the rule on the step completes without a give-up and is bit-identical to a step with no
    collective at all.
"""
import ctypes
import time

import pytest
import torch

from autovc_amd import _lib
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import onehot_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu

B, T = 256, 64  # config 4's per-rank batch: every decoder LSTM backward is a persistent launch
HOG_WG, HOG_LDS, HOG_US = 192, 160 * 1024, 300_000  # 192 of the 256 CUs for 300 ms
SPIN = 1 << 13


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class HogCollective:
    """all_reduce stand-in: the first `n_hogs` calls hold HOG_WG CUs for HOG_US on a side stream
    (ordered after the issuing stream, like an RCCL launch); later calls are empty."""

    def __init__(self, dev, n_hogs=2):
        self.dev = dev
        self.stream = torch.cuda.Stream(device=dev)
        self.left = n_hogs
        self.calls = 0

    def __call__(self, t):
        self.calls += 1
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))
        if self.left > 0:
            self.left -= 1
            _lib.call("avc_debug_hog", _lib.context(self.dev), HOG_WG, HOG_LDS, HOG_US, self.stream.cuda_stream)
            n, t0 = ctypes.c_int(0), time.time()
            while n.value < HOG_WG and time.time() - t0 < 20:  # the late peer: CUs held from now on
                _lib.call("avc_debug_hog_resident", _lib.context(self.dev), ctypes.byref(n))
                time.sleep(0.001)
            assert n.value == HOG_WG, f"only {n.value} of {HOG_WG} hog workgroups became resident"
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _Work(ev)


def _giveups():
    n = ctypes.c_long(0)
    _lib.call("avc_lstm_persist_status", ctypes.byref(n))
    return n.value


def _model(dev):
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    ae.to(dev).train()
    ae.configure_optimizer()
    return ae


def _batch(dev):
    X = torch.from_numpy(synthetic_mel(91, B, T)).to(dev)
    c = torch.from_numpy(onehot_embedding(B)).to(dev)
    return X, c


@pytest.fixture
def short_spins():
    _lib.call("avc_debug_persist_spin_limit", SPIN)
    yield
    _lib.call("avc_debug_persist_spin_limit", 0)


def test_plan_is_persistent():
    for H in (512, 1024):
        assert _lib.load().avc_bptt_persist_eligible(T, B, H) == 1


def test_unfenced_bptt_beside_held_cus_gives_up(cuda_device, short_spins):
    """Negative control: the rule off, a bucket's collective holds 192 CUs when the lstm2 BPTT
    dispatches -> the bounded waits give up (NaN gradients, update skipped, next call raises)."""
    X, c = _batch(cuda_device)
    warm = _model(cuda_device)  # first calls load code objects (hundreds of ms of host time)
    warm.train_step(X, c)
    warm.check_health()
    del warm
    ae = _model(cuda_device)
    hog = HogCollective(cuda_device)
    ae.grad_comm = dict(all_reduce=hog, world_size=1, co_residency=False)
    before = _giveups()
    keep = ae._flat_param.detach().clone()
    try:
        # a later persistent launch of the same backward may already report the give-up
        _, norm = ae.train_step(X, c)
        torch.cuda.synchronize()
        raised = False
    except RuntimeError as e:
        assert "abandoned a bounded wait" in str(e)
        raised = True
    torch.cuda.synchronize()
    assert hog.calls > 0
    assert _giveups() > before, "the BPTT completed although 192 CUs were held during its dispatch"
    assert torch.equal(keep, ae._flat_param)  # no NaN gradient was applied
    if not raised:
        assert not torch.isfinite(norm).item()
        with pytest.raises(RuntimeError, match="abandoned a bounded wait"):
            ae.check_health()


def test_fenced_bptt_completes_beside_held_cus(cuda_device, short_spins):
    """The rule on: the same held CUs, no give-up, and the step equals a step without any
    collective bit for bit (loss, grad norm, parameters, Adam moments, EMA)."""
    X, c = _batch(cuda_device)
    ref = _model(cuda_device)
    l0, n0 = ref.train_step(X, c)
    ref_state = [t.detach().clone() for t in (ref._flat_param, ref.optimiser.exp_avg, ref.optimiser.exp_avg_sq,
                                              ref.avg_params)]
    ref.check_health()
    del ref

    ae = _model(cuda_device)
    hog = HogCollective(cuda_device)
    ae.grad_comm = dict(all_reduce=hog, world_size=1)
    before = _giveups()
    launches = _lib.persist_launches(cuda_device)
    loss, norm = ae.train_step(X, c)
    torch.cuda.synchronize()
    assert _giveups() == before
    ae.check_health()
    # the lstm2 (2 layers) and lstm1 BPTTs ran persistent, every bucket went through the stand-in
    assert _lib.persist_launches(cuda_device) - launches >= 3
    assert hog.calls == len(ae._reducer.buckets) and hog.left == 0
    assert torch.equal(loss, l0) and torch.equal(norm, n0)
    for a, b in zip(ref_state, (ae._flat_param, ae.optimiser.exp_avg, ae.optimiser.exp_avg_sq, ae.avg_params)):
        assert torch.equal(a, b)
    # issue order: every bucket once, in index order
    assert [b for b, _ in ae._reducer.launch_log] == list(range(len(ae._reducer.buckets)))
