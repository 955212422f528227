"""Forward parity margin at C2 (B = 64, T = 128, train-mode BN as convert() runs it) over several
weight sets, not just the seed-0 Xavier init the golden fixtures use: two more seeds, the seed-0
matrices x4 and x0.25 (every parameter of rank >= 2: conv kernels, LSTM and Linear matrices), and
the weights after 20 GPU training steps (oracle run on those very weights).

For each set three distances are reported on mel / mel_post / codes:
  * GPU vs the oracle in fp32 (bit-identical to the reference: tests/golden) -- the north_star
    criterion, max|d| <= 1e-4;
  * GPU vs the oracle in float64 (exact arithmetic to ~1e-15);
  * the fp32 reference itself vs float64.
The reference's own distance from exact arithmetic is part of every GPU-vs-reference number (the
train-mode postnet BNs amplify input noise ~60x), so the GPU-vs-float64 column is what
says how good the HIP arithmetic is.  The test writes gpurun_out/r06_margin.json (copied to
profiles/r06_margin.json)."""
import json
import os

import numpy as np
import pytest
import torch

from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import onehot_embedding, synthetic_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu

TOL_MEL = 1e-4
B, T = 64, 128
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "r06_margin.json")


def _scaled(sd, f):
    return {k: (v * f if v.is_floating_point() and v.dim() >= 2 else v.clone()) for k, v in sd.items()}


def _trained(dev, steps=20):
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    ae.to(dev).train()
    ae.configure_optimizer()
    for s in range(steps):
        X = torch.from_numpy(synthetic_mel(700 + s, B, T)).to(dev)
        c = torch.from_numpy(onehot_embedding(B, offset=3 * s)).to(dev)
        ae.train_step(X, c)
    ae.check_health()
    return {k: v.detach().cpu().clone() for k, v in ae.state_dict().items()}


WEIGHT_SETS = ["seed0", "seed1", "seed2", "seed0_x4", "seed0_x0.25", "trained20"]


@pytest.fixture(scope="module")
def results():
    res = {}
    yield res
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as fh:
        json.dump(res, fh, indent=1)


def _weights(dev, name):
    if name.startswith("seed") and "_x" not in name:
        return torch_state_dict(int(name[4:]))
    if name == "seed0_x4":
        return _scaled(torch_state_dict(0), 4.0)
    if name == "seed0_x0.25":
        return _scaled(torch_state_dict(0), 0.25)
    return _trained(dev)


def _margin(dev, results, key, sd, B, T, xseed=1, strict=False):
    """GPU forward vs the oracle in fp32 and float64 (see the module docstring); records and checks.
    strict: the 1e-4 bar is asserted whatever the reference's own distance from float64 (the
    batches convert() runs)."""
    from oracle import autovc_oracle as orc
    torch.set_num_threads(min(16, torch.get_num_threads()))
    x = synthetic_mel(xseed, B, T)
    co, ct = synthetic_embedding(101, B), synthetic_embedding(201, B)
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(sd)
    ae.to(dev).train()
    with torch.no_grad():
        outs = [o.cpu() for o in ae(*(torch.from_numpy(a).to(dev) for a in (x, co, ct)))]
    ae.check_health()

    def oracle(dtype):
        s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        bufs = {k: v for k, v in s.items() if "running" in k or "num_batches" in k}
        with torch.no_grad():
            return orc.forward(s, *(torch.from_numpy(a).to(dtype) for a in (x, co, ct)), True, bufs)
    r32, r64 = oracle(torch.float32), oracle(torch.float64)
    rec = {"B": B, "T": T}
    for i, k in enumerate(("mel", "mel_post", "codes")):
        g, a, e = outs[i].double(), r32[i].double(), r64[i]
        rec[k] = {"gpu_vs_ref": float((g - a).abs().max()), "gpu_vs_f64": float((g - e).abs().max()),
                  "ref_vs_f64": float((a - e).abs().max()), "max_abs": float(e.abs().max())}
    worst = max(rec[k]["gpu_vs_ref"] for k in ("mel", "mel_post", "codes"))
    rec["margin"] = TOL_MEL / worst if worst > 0 else float("inf")
    results[key] = rec
    print(f"{key}: " + "; ".join(f"{k} gpu-ref {v['gpu_vs_ref']:.2e} gpu-f64 {v['gpu_vs_f64']:.2e} "
                                 f"ref-f64 {v['ref_vs_f64']:.2e}" for k, v in rec.items() if isinstance(v, dict))
          + f"; margin {rec['margin']:.2f}x")
    assert np.isfinite(worst)
    for k in ("mel", "mel_post", "codes"):
        r = rec[k]
        # the HIP arithmetic is not further from exact than the fp32 reference's own (factor 2 and
        # a 1e-7 floor: both are sums of many roundings of either sign)
        assert r["gpu_vs_f64"] <= 2 * r["ref_vs_f64"] + 1e-7, (k, r)
        # north_star's 1e-4 bar is asserted where the fp32 reference itself stays within half of it
        # from exact arithmetic.  Where it does not (the x4 / x0.25 sets: ref - f64 1.5e-3 / 1.5e-4)
        # the bar is NOT met (GPU - ref 2.5e-3 / 1.6e-4), and only the line above is checked: the GPU
        # is closer to float64 than the reference there, so the distance is the reference's own
        # rounding, which an implementation with a different summation order cannot reproduce.
        if strict or r["ref_vs_f64"] < TOL_MEL / 2:
            assert r["gpu_vs_ref"] <= TOL_MEL, (k, r)
    return rec


# the batch sizes convert() actually runs (voice_converter.py:171-175: one utterance, B = 1, with
# cut=False; batch_forward's slices otherwise) and the smoke test's B = 2, T = 64
SMALL = [(0, 1, 128), (1, 1, 128), (2, 1, 128), (0, 1, 300), (0, 2, 64), (1, 2, 64), (0, 2, 128), (2, 3, 96)]
# convert(cut=False) runs one utterance at its full length: B = 1 at T = 1024 and 2000
SMALL += [(s, 1, t) for t in (1024, 2000) for s in (0, 1, 2)]


@pytest.mark.parametrize("seed,B,T", SMALL, ids=[f"seed{s}_B{b}_T{t}" for s, b, t in SMALL])
def test_small_batch_margin(cuda_device, results, seed, B, T):
    _margin(cuda_device, results, f"seed{seed}_B{B}_T{T}", torch_state_dict(seed), B, T, xseed=5 + seed, strict=True)


@pytest.mark.parametrize("name", WEIGHT_SETS)
def test_c2_forward_margin(cuda_device, results, name):
    _margin(cuda_device, results, name, _weights(cuda_device, name), B, T)
