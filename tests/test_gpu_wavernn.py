"""WaveRNN vocoder `generate` on the GPU through the C ABI.

Pins:
* up-sampling and the teacher-forced network against the reference class's own outputs
  (tests/golden/wavernn_ref.npz): max |Δ| <= 2e-5 on the mel / aux features, <= 1e-4 on logits
  (fp32, K = 512..544 dot products in a different order than oneDNN's);
* sampling: the reference draws from torch's RNG, so parity is distribution-level.  Our sampler
  and the oracle share one counter-based uniform stream, so (a) with the network's output held
  fixed (fc3 weight = 0) every sample must equal the oracle's to fp32 rounding, and their
  distribution must match the mixture-of-logistics law (Kolmogorov–Smirnov); (b) the first
  steps of a full generation follow the oracle's trajectory sample for sample;
* the cross-fade / fade-out (float64 like the reference's numpy) bit-for-bit against the oracle
  on the GPU's own samples."""
import math

import numpy as np
import pytest
import torch

from autovc_amd.weights import synthetic_mel, wavernn_state_dict
from autovc_amd.wavernn import WaveRNN
from oracle import wavernn_oracle as wo
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sd():
    return wavernn_state_dict(0)


def make(dev, sd, mode="MOL"):
    net = WaveRNN(device=dev, mode=mode)
    net.load_state_dict({k: v for k, v in sd.items()})
    net.eval()
    return net


def test_upsample_matches_reference(cuda_device, sd):
    g = load_golden("wavernn_ref")
    net = make(cuda_device, sd)
    m, aux = net.upsample_features(torch.from_numpy(g["up_mel_in"]))
    torch.cuda.synchronize()
    em = np.abs(m.cpu().numpy() - g["up_m"][0]).max()
    aux_up = np.repeat(aux.cpu().numpy(), net.hop_length, axis=0)
    ea = np.abs(aux_up - g["up_aux"][0]).max()
    print(f"upsample: max|d m| {em:.2e}, max|d aux| {ea:.2e}")
    assert em <= 2e-5 and ea <= 2e-5


@pytest.mark.parametrize("row", [0, 1])
def test_teacher_forced_network_matches_reference(cuda_device, sd, row):
    g = load_golden("wavernn_ref")
    net = make(cuda_device, sd)
    logits = net(torch.from_numpy(g["fwd_x"][row:row + 1]), torch.from_numpy(g["fwd_mels"][row:row + 1]))
    torch.cuda.synchronize()
    err = np.abs(logits.cpu().numpy()[0] - g["fwd_logits"][row]).max()
    print(f"teacher-forced logits row {row}: max|d| {err:.2e} over {g['fwd_logits'].shape[1]} steps")
    assert err <= 1e-4


def _mol_cdf(x, pi, mu, s):
    return sum(p / (1.0 + math.exp(-(x - m) / sc)) for p, m, sc in zip(pi, mu, s))


@pytest.mark.parametrize("mode", ["MOL", "RAW"])
def test_sampler_matches_oracle_and_law(cuda_device, sd, mode):
    """fc3.weight = 0: the logits are fc3.bias at every step, so samples are i.i.d. draws of one
    distribution; GPU == oracle draw for draw, and the empirical law matches the analytic one."""
    sdm = dict(sd)
    nc = 30 if mode == "MOL" else 18
    rng = np.random.default_rng(5)
    bias = rng.uniform(-1, 1, nc).astype(np.float32)
    if mode == "MOL":
        bias[10:20] = np.linspace(-0.6, 0.6, 10)   # means
        bias[20:30] = rng.uniform(-4, -2, 10)      # log scales
    sdm["fc3.weight"] = torch.zeros(nc, 512)
    sdm["fc3.bias"] = torch.from_numpy(bias)
    net = make(cuda_device, sdm, mode)
    mel = torch.from_numpy(synthetic_mel(9, 1, 24))
    seed = 1234567
    samples, _, _ = net._run(mel, True, 200, 20, seed)
    torch.cuda.synchronize()
    s = samples.cpu().numpy()
    rows = np.arange(s.shape[0])
    lg = torch.from_numpy(np.tile(bias, (s.shape[0], 1)))
    ref = np.zeros_like(s)
    for i in range(s.shape[1]):
        if mode == "MOL":
            u = torch.from_numpy(wo.uniforms(seed, rows, i, 11))
            ref[:, i] = wo.sample_mol(lg, u[:, :10], u[:, 10]).numpy()
        else:
            u = torch.from_numpy(wo.uniforms(seed, rows, i, 1))
            ref[:, i] = wo.sample_raw(lg, u[:, 0]).numpy()
    err = np.abs(s - ref).max()
    print(f"{mode}: {s.size} draws, max|GPU - oracle| {err:.2e}")
    if mode == "MOL":
        assert err <= 2e-6
    else:  # a uniform within fp32 rounding of a CDF step may land one class apart
        assert (s != ref).sum() <= 1
    x = np.sort(s.ravel().astype(np.float64))
    n = x.size
    if mode == "MOL":
        pi = np.exp(bias[:10] - bias[:10].max())
        pi /= pi.sum()
        mu, sc = bias[10:20].astype(np.float64), np.exp(np.maximum(bias[20:30], np.log(1e-14))).astype(np.float64)
        inner = (x > -1) & (x < 1)
        F = np.array([_mol_cdf(v, pi, mu, sc) for v in x[inner]])
        emp = (np.arange(n)[inner] + 1) / n
        ks = np.abs(emp - F).max()
        print(f"MOL KS distance {ks:.4f} (n = {n})")
        assert ks < 1.63 / math.sqrt(n) + 2e-3  # 1% critical value
    else:
        p = np.exp(bias - bias.max())
        p /= p.sum()
        k = np.rint((x + 1.0) * (nc - 1) / 2.0).astype(int)
        counts = np.bincount(k, minlength=nc)
        chi2 = ((counts - n * p) ** 2 / (n * p)).sum()
        print(f"RAW chi2 {chi2:.1f} over {nc} classes (n = {n})")
        assert chi2 < 40.8  # 99.9% quantile, 17 dof


def test_generate_follows_oracle_then_crossfades_exactly(cuda_device, sd):
    net = make(cuda_device, sd)
    mel = torch.from_numpy(synthetic_mel(11, 1, 24))
    seed = 99
    target, overlap = 1000, 100
    samples, _, wave = net._run(mel, True, target, overlap, seed)
    torch.cuda.synchronize()
    s = samples.cpu().numpy()
    steps = 48
    ref = wo.generate({k: v for k, v in sd.items()}, mel, batched=True, target=target, overlap=overlap, seed=seed,
                      steps=steps)
    err = np.abs(s[:, :steps] - ref).max()
    print(f"generate: {s.shape[0]} fold rows, first {steps} steps max|GPU - oracle| {err:.2e}")
    assert err <= 1e-4
    assert np.isfinite(s).all() and np.abs(s).max() <= 1.0
    # the cross-fade / fade-out of the GPU's own samples, float64 like the reference
    y = wo.xfade_and_unfold(s.astype(np.float64), target, overlap)
    wave_len = (mel.shape[-1] - 1) * wo.HOP
    y = y[:wave_len]
    y[-20 * wo.HOP:] *= np.linspace(1, 0, 20 * wo.HOP)
    got = wave.cpu().numpy()
    assert got.shape == (wave_len,)
    np.testing.assert_array_equal(got, y.astype(np.float32))


def test_generate_api(cuda_device, sd):
    """The reference call shape: generate(mel (1, 80, T)) -> np.float32 of (T - 1) * hop, seeded
    by torch's RNG (reproducible under torch.manual_seed, different otherwise)."""
    net = make(cuda_device, sd)
    mel = torch.from_numpy(synthetic_mel(12, 1, 48)).to(cuda_device)
    torch.manual_seed(3)
    a = net.generate(mel)
    torch.manual_seed(3)
    b = net.generate(mel)
    c = net.generate(mel)
    assert a.dtype == np.float32 and a.shape == ((48 - 1) * 275,)
    np.testing.assert_array_equal(a, b)
    assert not np.array_equal(a, c)
    assert np.isfinite(a).all() and np.abs(a).max() <= 1.0
    with pytest.raises(ValueError):
        net.generate(mel[..., :10])
