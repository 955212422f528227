"""Dead h stores of the persistent recurrences inside the whole-Generator forward
(avc_dead_h_stores, autovc_hip_debug.h).

lstm2's layer-0 h is handed to layer 1 only as the split hand-off, and lstm1's / lstm2's last
layer is read by the next contraction only as its split image: the fp32 h stores of those are
skipped by default.  Outputs must not change, eager, captured and replayed."""
import pytest
import torch

from autovc_amd import _lib
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu


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


@pytest.mark.parametrize("B,T", [(64, 128), (32, 96), (3, 40)])
def test_dead_h_stores_leave_outputs_unchanged(cuda_device, B, T):
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
