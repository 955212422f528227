"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of the WaveRNN vocoder's `generate` (SURVEY §8f row 4,
autovc/wavernn/model.py:214-329, autovc/wavernn/distribution.py:87-123), in torch-CPU fp32 for
the network and float64 numpy for the fold / cross-fade arithmetic, as the reference does.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Sampling: the reference draws its uniforms from torch's global RNG (distribution.py:103,113),
which no other implementation can reproduce.  Generation here takes its uniforms from a
counter-based stream instead (`uniforms`, the same hash the HIP kernels use), so the oracle and
the GPU path draw identical noise and their outputs can be compared sample for sample; against
the reference the sampler is pinned by feeding the reference's own uniforms back in
(tests/golden/make_golden_wavernn.py records them with torch.manual_seed), and the rest of the
network by the reference's teacher-forced `forward` (model.py:180-211).

Paths relative to /root/reference.
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn.functional as F

HOP = 275                        # hparams.py:96
UPSAMPLE = (5, 5, 11)            # hparams.py:102
PAD = 2                          # hparams.py:104
RES_BLOCKS = 10                  # hparams.py:105
LOG_SCALE_MIN = float(np.log(1e-14))  # distribution.py:96-97

_GOLDEN = 0x9E3779B97F4A7C15
_MASK = (1 << 64) - 1


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniforms(seed: int, rows: np.ndarray, step: int, draws: int) -> np.ndarray:
    """float32 [len(rows)][draws] in [1e-5, 1 - 1e-5] (the reference's uniform_(1e-5, 1 - 1e-5)
    range, distribution.py:103,113): splitmix64 of the counter (row << 40 | step << 8 | draw)
    offset by the seed, top 24 bits, then lo + span * u in two fp32 roundings."""
    with np.errstate(over="ignore"):
        base = _mix(np.array([((seed + 1) * _GOLDEN) & _MASK], dtype=np.uint64))[0]
        ctr = ((rows.astype(np.uint64)[:, None] << np.uint64(40)) | (np.uint64(step) << np.uint64(8)) |
               np.arange(draws, dtype=np.uint64)[None, :])
        z = _mix(ctr * np.uint64(_GOLDEN) + base)
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))
    return np.float32(1e-5) + np.float32(0.99998) * u


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.1, 1e-5)


def upsample(sd: Dict[str, torch.Tensor], mels: torch.Tensor, res_blocks: int = RES_BLOCKS,
             factors=UPSAMPLE, pad: int = PAD) -> Tuple[torch.Tensor, torch.Tensor]:
    """UpsampleNetwork.forward (model.py:66-93) in eval mode (generate() calls self.eval()):
    MelResNet (conv_in k=2pad+1 no bias -> BN -> relu -> res_blocks x [1x1 conv, BN, relu, 1x1
    conv, BN, + residual] -> 1x1 conv_out with bias, model.py:34-49), stretched x prod(factors);
    the mel through Stretch2d + Conv2d(1, 1, (1, 2s+1), padding (0, s)) per factor, then cropped
    by pad * prod(factors) on both sides.  mels (B, 80, T) -> ((B, L, 80), (B, L, 128))."""
    p = "upsample.resnet."
    x = F.conv1d(mels, sd[p + "conv_in.weight"])
    x = F.relu(_bn(x, sd, p + "batch_norm"))
    for i in range(res_blocks):
        q = f"{p}layers.{i}."
        r = x
        x = F.relu(_bn(F.conv1d(x, sd[q + "conv1.weight"]), sd, q + "batch_norm1"))
        x = _bn(F.conv1d(x, sd[q + "conv2.weight"]), sd, q + "batch_norm2") + r
    aux = F.conv1d(x, sd[p + "conv_out.weight"], sd[p + "conv_out.bias"])
    total = int(np.prod(factors))
    aux = aux.repeat_interleave(total, dim=2)
    m = mels.unsqueeze(1)
    for j, s in enumerate(factors):
        m = m.repeat_interleave(s, dim=3)
        m = F.conv2d(m, sd[f"upsample.up_layers.{2 * j + 1}.weight"], padding=(0, s))
    indent = pad * total
    m = m.squeeze(1)[:, :, indent:-indent]
    return m.transpose(1, 2), aux.transpose(1, 2)


def pad_tensor(x: torch.Tensor, pad: int, side: str = "both") -> torch.Tensor:
    """model.py:284-294: zero padding along dim 1 of (B, T, C)."""
    b, t, c = x.size()
    total = t + 2 * pad if side == "both" else t + pad
    out = torch.zeros(b, total, c, dtype=x.dtype)
    if side in ("before", "both"):
        out[:, pad:pad + t, :] = x
    elif side == "after":
        out[:, :t, :] = x
    return out


def fold_with_overlap(x: torch.Tensor, target: int, overlap: int) -> torch.Tensor:
    """model.py:296-339."""
    _, total_len, features = x.size()
    num_folds = (total_len - overlap) // (target + overlap)
    extended_len = num_folds * (overlap + target) + overlap
    remaining = total_len - extended_len
    if remaining != 0:
        num_folds += 1
        x = pad_tensor(x, target + 2 * overlap - remaining, side="after")
    folded = torch.zeros(num_folds, target + 2 * overlap, features, dtype=x.dtype)
    for i in range(num_folds):
        s = i * (target + overlap)
        folded[i] = x[0, s:s + target + 2 * overlap, :]
    return folded


def xfade_and_unfold(y: np.ndarray, target: int, overlap: int) -> np.ndarray:
    """model.py:341-399 (float64)."""
    y = np.array(y, dtype=np.float64)
    num_folds, length = y.shape
    target = length - 2 * overlap
    total_len = num_folds * (target + overlap) + overlap
    silence_len = overlap // 2
    fade_len = overlap - silence_len
    t = np.linspace(-1, 1, fade_len, dtype=np.float64)
    fade_in = np.concatenate([np.zeros(silence_len), np.sqrt(0.5 * (1 + t))])
    fade_out = np.concatenate([np.ones(silence_len), np.sqrt(0.5 * (1 - t))])
    y[:, :overlap] *= fade_in
    y[:, -overlap:] *= fade_out
    out = np.zeros(total_len, dtype=np.float64)
    for i in range(num_folds):
        s = i * (target + overlap)
        out[s:s + target + 2 * overlap] += y[i]
    return out


def _gru(x, h, sd, p):
    """nn.GRU / nn.GRUCell (gate order r, z, n): r = σ(W_ir x + b_ir + W_hr h + b_hr), z likewise,
    n = tanh(W_in x + b_in + r ⊙ (W_hn h + b_hn)), h' = (1 - z) ⊙ n + z ⊙ h."""
    gi = F.linear(x, sd[p + ".weight_ih_l0"], sd[p + ".bias_ih_l0"])
    gh = F.linear(h, sd[p + ".weight_hh_l0"], sd[p + ".bias_hh_l0"])
    H = h.shape[-1]
    r = torch.sigmoid(gi[..., :H] + gh[..., :H])
    z = torch.sigmoid(gi[..., H:2 * H] + gh[..., H:2 * H])
    n = torch.tanh(gi[..., 2 * H:] + r * gh[..., 2 * H:])
    return (1 - z) * n + z * h


def step(sd, x_prev, m_t, a_t, h1, h2):
    """One generate step up to the logits (model.py:263-284).  x_prev (R, 1), m_t (R, 80),
    a_t (R, 128) -> logits (R, n_classes), h1, h2."""
    d = a_t.shape[-1] // 4
    a1, a2, a3, a4 = (a_t[:, d * i:d * (i + 1)] for i in range(4))
    x = F.linear(torch.cat([x_prev, m_t, a1], dim=1), sd["I.weight"], sd["I.bias"])
    h1 = _gru(x, h1, sd, "rnn1")
    x = x + h1
    h2 = _gru(torch.cat([x, a2], dim=1), h2, sd, "rnn2")
    x = x + h2
    x = F.relu(F.linear(torch.cat([x, a3], dim=1), sd["fc1.weight"], sd["fc1.bias"]))
    x = F.relu(F.linear(torch.cat([x, a4], dim=1), sd["fc2.weight"], sd["fc2.bias"]))
    return F.linear(x, sd["fc3.weight"], sd["fc3.bias"]), h1, h2


def forward(sd, x: torch.Tensor, mels: torch.Tensor) -> torch.Tensor:
    """WaveRNN.forward (model.py:180-211), the teacher-forced network: x (B, L) previous samples,
    mels (B, 80, T) -> logits (B, L, n_classes), L = (T - 2 pad) * hop."""
    m, aux = upsample(sd, mels)
    B, L, _ = m.shape
    R = sd["rnn1.weight_hh_l0"].shape[1]
    h1 = torch.zeros(B, R)
    h2 = torch.zeros(B, R)
    out = []
    for i in range(L):
        logits, h1, h2 = step(sd, x[:, i:i + 1], m[:, i], aux[:, i], h1, h2)
        out.append(logits)
    return torch.stack(out, dim=1)


def sample_mol(logits: torch.Tensor, u_mix: torch.Tensor, u_log: torch.Tensor) -> torch.Tensor:
    """sample_from_discretized_mix_logistic (distribution.py:87-123) with its two uniform draws
    given: u_mix (R, nr_mix) for the Gumbel-max mixture choice, u_log (R,) for the logistic."""
    nr = logits.shape[1] // 3
    temp = logits[:, :nr] - torch.log(-torch.log(u_mix))
    k = temp.argmax(dim=1)
    one_hot = F.one_hot(k, nr).float()
    means = torch.sum(logits[:, nr:2 * nr] * one_hot, dim=-1)
    log_scales = torch.clamp(torch.sum(logits[:, 2 * nr:3 * nr] * one_hot, dim=-1), min=LOG_SCALE_MIN)
    x = means + torch.exp(log_scales) * (torch.log(u_log) - torch.log(1.0 - u_log))
    return torch.clamp(torch.clamp(x, min=-1.0), max=1.0)


def sample_raw(logits: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """model.py:310-315: Categorical(softmax(logits)) by inverse CDF on one uniform, mapped to
    2 k / (n_classes - 1) - 1."""
    p = torch.softmax(logits, dim=1)
    cdf = torch.cumsum(p, dim=1)
    k = torch.clamp((cdf < u[:, None]).sum(dim=1), max=logits.shape[1] - 1)
    return 2.0 * k.float() / (logits.shape[1] - 1.0) - 1.0


def generate(sd, mel: torch.Tensor, batched=True, target=11_000, overlap=550, mode="MOL", seed=0,
             steps=None):
    """WaveRNN.generate (model.py:214-329) with the counter-based uniforms above.  Returns the
    float32 waveform; `steps` (testing) stops the sequential loop early and returns the raw
    per-row samples (R, steps) instead."""
    with torch.no_grad():
        wave_len = (mel.size(-1) - 1) * HOP
        m = pad_tensor(mel.transpose(1, 2), pad=PAD, side="both")
        m, aux = upsample(sd, m.transpose(1, 2))
        if batched:
            m = fold_with_overlap(m, target, overlap)
            aux = fold_with_overlap(aux, target, overlap)
        R_, L, _ = m.shape
        H = sd["rnn1.weight_hh_l0"].shape[1]
        h1 = torch.zeros(R_, H)
        h2 = torch.zeros(R_, H)
        x = torch.zeros(R_, 1)
        rows = np.arange(R_)
        n = L if steps is None else min(steps, L)
        out = np.zeros((R_, n), dtype=np.float32)
        for i in range(n):
            logits, h1, h2 = step(sd, x, m[:, i], aux[:, i], h1, h2)
            if mode == "MOL":
                u = torch.from_numpy(uniforms(seed, rows, i, logits.shape[1] // 3 + 1))
                s = sample_mol(logits, u[:, :-1], u[:, -1])
            else:
                u = torch.from_numpy(uniforms(seed, rows, i, 1))
                s = sample_raw(logits, u[:, 0])
            out[:, i] = s.numpy()
            x = s[:, None]
        if steps is not None:
            return out
    output = out.astype(np.float64)
    output = xfade_and_unfold(output, target, overlap) if batched else output[0]
    fade_out = np.linspace(1, 0, 20 * HOP)
    output = output[:wave_len]
    output[-20 * HOP:] *= fade_out
    return output.astype(np.float32)
