"""Training-loss curve at BASELINE config 3 (B = 256, T = 128) against the reference's own learn()
(autovc/auto_encoder/model.py:218-361): 12 steps of AutoEncoder.train_step on the seeded batches
of tests/golden/train_b256_t128_curve.npz (tests/golden/make_golden.py: curve_case), per-step loss
and pre-clip gradient norm.

Tolerance.  A training trajectory is chaotic in rounding noise: Adam's first steps move every
weight by about lr * sign(g), and the elements with g ~ 0 take noise signs.  The fixture carries
the same 12 steps in float64 (the oracle's Trainer, exact to ~1e-15): the fp32 reference itself
leaves that curve by up to 1.9 % in loss and 12 % in gradient norm by step 8-11.  So at step s the
GPU must stay within  k * E(s) + floor  of the reference, where E(s) = max over s' <= s of the
reference's relative distance from float64 (the spread any correct fp32 implementation has by then),
k = 2, floor = 2e-5 (loss) / 2e-3 (grad norm: the first step, one backward apart).  Step 1 is
one forward + backward from identical weights and is held much tighter than the envelope (1e-5
relative loss, 2e-3 relative norm).  The mean loss of the 12 steps must agree to 0.5 %."""
import os

import numpy as np
import pytest
import torch

from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import onehot_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "train_b256_t128_curve.npz")


def test_c3_loss_curve_against_reference_learn(cuda_device):
    d = np.load(FIX)
    B, T = int(d["B"]), int(d["T"])
    seeds, offs = d["seeds"], d["onehot_offsets"]
    ae = AutoEncoder(device=cuda_device, verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    ae.to(cuda_device).train()
    ae.configure_optimizer()
    losses, norms = [], []
    for s in range(len(seeds)):
        X = torch.from_numpy(synthetic_mel(int(seeds[s]), B, T)).to(cuda_device)
        c = torch.from_numpy(onehot_embedding(B, offset=int(offs[s]))).to(cuda_device)
        loss, norm = ae.train_step(X, c)
        losses.append(float(loss))
        norms.append(float(norm))
    ae.check_health()
    losses, norms = np.array(losses), np.array(norms)
    ref_l, ref_n, f64_l, f64_n = d["losses"], d["grad_norms"], d["losses_f64"], d["grad_norms_f64"]
    rel = lambda a, b: np.abs(a - b) / np.abs(b)  # noqa: E731
    env_l = np.maximum.accumulate(rel(ref_l, f64_l))
    env_n = np.maximum.accumulate(rel(ref_n, f64_n))
    for s in range(len(seeds)):
        print(f"step {s + 1:2d}: loss {losses[s]:.7f} ref {ref_l[s]:.7f} f64 {f64_l[s]:.7f} "
              f"(gpu-ref {rel(losses[s], ref_l[s]):.1e}, ref-f64 {rel(ref_l[s], f64_l[s]):.1e}, "
              f"gpu-f64 {rel(losses[s], f64_l[s]):.1e}) | norm {norms[s]:.6f} ref {ref_n[s]:.6f} "
              f"f64 {f64_n[s]:.6f} (gpu-ref {rel(norms[s], ref_n[s]):.1e}, ref-f64 {rel(ref_n[s], f64_n[s]):.1e})")
    assert np.all(np.isfinite(losses)) and np.all(np.isfinite(norms))
    assert rel(losses[0], ref_l[0]) <= 1e-5
    assert rel(norms[0], ref_n[0]) <= 2e-3
    assert np.all(rel(losses, ref_l) <= 2 * env_l + 2e-5), rel(losses, ref_l)
    assert np.all(rel(norms, ref_n) <= 2 * env_n + 2e-3), rel(norms, ref_n)
    assert abs(losses.mean() - ref_l.mean()) / ref_l.mean() <= 5e-3
