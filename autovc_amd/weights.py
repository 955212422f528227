"""Seeded synthetic weights for the AutoVC Generator (no checkpoints are reachable offline).

A counter-based splitmix64 stream per tensor gives bit-identical weights on every host and
numpy version, so fixtures only need to record the seed.  Bounds follow the reference init
(SURVEY §8a row a1):

* Conv1d weight: xavier_uniform with gain relu=sqrt(2) for encoder/decoder convs
  (autovc/auto_encoder/encoder.py:41-45, decoder.py:43-47), tanh=5/3 for postnet 0-3 and
  linear=1 for postnet 4 (postnet.py:21-47); ConvNorm in net_layers.py:44-45.
* Linear weight (decoder.linear_projection): xavier_uniform gain 1 (net_layers.py:15-17).
* Conv/Linear bias: PyTorch default U(+-1/sqrt(fan_in)).
* LSTM weights and biases: PyTorch default U(+-1/sqrt(H)).
* BatchNorm: the reference starts at gamma=1, beta=0, running (0, 1).  With
  ``bn_perturb=True`` (the default for tests/bench) gamma, beta and the running statistics are
  drawn from small ranges instead so that affine/eval-mode bugs cannot hide behind identities.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def uniform01(seed: int, stream: int, n: int) -> np.ndarray:
    """n float64 values in [0,1) with 24 random bits each, from (seed, stream)."""
    with np.errstate(over="ignore"):
        base = _mix(np.array([(seed * 1_000_003 + stream + 1) & 0xFFFFFFFFFFFFFFFF],
                             dtype=np.uint64) * _GOLDEN)[0]
        ctr = np.arange(1, n + 1, dtype=np.uint64) * _GOLDEN + base
        z = _mix(ctr)
    return (z >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))


def _u(seed, stream, shape, lo, hi) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    v = lo + (hi - lo) * uniform01(seed, stream, n)
    return v.astype(np.float32).reshape(shape)


def param_specs(dim_neck=32, dim_emb=256, dim_pre=512):
    """(name, shape, kind, extra) in the reference state_dict order."""
    specs = []
    gain_relu, gain_tanh, gain_lin = math.sqrt(2.0), 5.0 / 3.0, 1.0

    def conv(prefix, cin, cout, gain):
        specs.append((prefix + ".0.conv.weight", (cout, cin, 5), "xavier", (gain, cin * 5, cout * 5)))
        specs.append((prefix + ".0.conv.bias", (cout,), "fanin", cin * 5))
        specs.append((prefix + ".1.weight", (cout,), "bn_gamma", None))
        specs.append((prefix + ".1.bias", (cout,), "bn_beta", None))
        specs.append((prefix + ".1.running_mean", (cout,), "bn_rmean", None))
        specs.append((prefix + ".1.running_var", (cout,), "bn_rvar", None))
        specs.append((prefix + ".1.num_batches_tracked", (), "bn_count", None))

    def lstm(prefix, din, h, layers, bidir):
        for l in range(layers):
            for sfx in ([""] + (["_reverse"] if bidir else [])):
                lin = din if l == 0 else h * (2 if bidir else 1)
                specs.append((f"{prefix}.weight_ih_l{l}{sfx}", (4 * h, lin), "lstm", h))
                specs.append((f"{prefix}.weight_hh_l{l}{sfx}", (4 * h, h), "lstm", h))
                specs.append((f"{prefix}.bias_ih_l{l}{sfx}", (4 * h,), "lstm", h))
                specs.append((f"{prefix}.bias_hh_l{l}{sfx}", (4 * h,), "lstm", h))

    for i in range(3):
        conv(f"encoder.convolutions.{i}", 80 + dim_emb if i == 0 else 512, 512, gain_relu)
    lstm("encoder.lstm", 512, dim_neck, 2, True)
    lstm("decoder.lstm1", dim_neck * 2 + dim_emb, dim_pre, 1, False)
    for i in range(3):
        conv(f"decoder.convolutions.{i}", dim_pre, dim_pre, gain_relu)
    lstm("decoder.lstm2", dim_pre, 1024, 2, False)
    specs.append(("decoder.linear_projection.linear_layer.weight", (80, 1024), "xavier", (gain_lin, 1024, 80)))
    specs.append(("decoder.linear_projection.linear_layer.bias", (80,), "fanin", 1024))
    conv("postnet.convolutions.0", 80, 512, gain_tanh)
    for i in range(1, 4):
        conv(f"postnet.convolutions.{i}", 512, 512, gain_tanh)
    conv("postnet.convolutions.4", 512, 80, gain_lin)
    return specs


def synthetic_state_dict(seed: int = 0, bn_perturb: bool = True, **dims) -> "OrderedDict[str, np.ndarray]":
    """Deterministic numpy state dict with the reference's keys, shapes and init bounds."""
    out = OrderedDict()
    for idx, (name, shape, kind, extra) in enumerate(param_specs(**dims)):
        if kind == "xavier":
            gain, fi, fo = extra
            a = gain * math.sqrt(6.0 / (fi + fo))
            out[name] = _u(seed, idx, shape, -a, a)
        elif kind == "fanin":
            b = 1.0 / math.sqrt(extra)
            out[name] = _u(seed, idx, shape, -b, b)
        elif kind == "lstm":
            b = 1.0 / math.sqrt(extra)
            out[name] = _u(seed, idx, shape, -b, b)
        elif kind == "bn_gamma":
            out[name] = _u(seed, idx, shape, 0.5, 1.5) if bn_perturb else np.ones(shape, np.float32)
        elif kind == "bn_beta":
            out[name] = _u(seed, idx, shape, -0.2, 0.2) if bn_perturb else np.zeros(shape, np.float32)
        elif kind == "bn_rmean":
            out[name] = _u(seed, idx, shape, -0.1, 0.1) if bn_perturb else np.zeros(shape, np.float32)
        elif kind == "bn_rvar":
            out[name] = _u(seed, idx, shape, 0.5, 1.5) if bn_perturb else np.ones(shape, np.float32)
        elif kind == "bn_count":
            out[name] = np.array(0, dtype=np.int64)
        else:  # pragma: no cover
            raise AssertionError(kind)
    return out


def torch_state_dict(seed: int = 0, bn_perturb: bool = True, device="cpu", **dims):
    import torch
    return OrderedDict((k, torch.from_numpy(v).to(device)) for k, v in
                       synthetic_state_dict(seed, bn_perturb, **dims).items())


def state_checksum(sd) -> float:
    """Order-sensitive float64 checksum used by fixtures to detect generator drift."""
    s = 0.0
    for i, (k, v) in enumerate(sd.items()):
        a = np.asarray(v.cpu().numpy() if hasattr(v, "cpu") else v, dtype=np.float64).ravel()
        if a.size:
            s += (i + 1) * float(a.sum()) + float((a * np.arange(1, a.size + 1) % 7).sum()) * 1e-6
    return s


# ---- synthetic inputs -------------------------------------------------------

def synthetic_mel(seed: int, B: int, T: int, n_mels: int = 80) -> np.ndarray:
    """U[0,1) mels, shape (B, 80, T): real mels are clipped to [0,1] (spectrogram.py:31)."""
    return _u(seed, 10_000_001, (B, n_mels, T), 0.0, 1.0)


def synthetic_embedding(seed: int, B: int, dim: int = 256) -> np.ndarray:
    """|N(0,1)| then L2-normalised, mimicking the speaker encoder's ReLU + L2 (model.py:85-88)."""
    u1 = uniform01(seed, 20_000_003, B * dim)
    u2 = uniform01(seed, 20_000_005, B * dim)
    g = np.abs(np.sqrt(-2.0 * np.log1p(-u1)) * np.cos(2 * np.pi * u2)).reshape(B, dim)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    return g.astype(np.float32)


def onehot_embedding(B: int, dim: int = 256, offset: int = 0) -> np.ndarray:
    """One-hot speaker ids c[i, i mod 256] = 1 as in dataloader.py:82-85."""
    c = np.zeros((B, dim), np.float32)
    c[np.arange(B), (np.arange(B) + offset) % dim] = 1.0
    return c


# ---- speaker encoder ---------------------------------------------------

def speaker_encoder_state_dict(seed: int = 0, n_in: int = 40, H: int = 256, E: int = 256, layers: int = 3,
                               device="cpu"):
    """SpeakerEncoder.state_dict() keys/shapes (speaker_encoder/model.py:48-57) with PyTorch's
    default init bounds: LSTM U(±1/√H), Linear U(±1/√fan_in)."""
    import torch
    out = OrderedDict()
    k = 1.0 / np.sqrt(H)
    stream = 50_000_000
    for l in range(layers):
        din = n_in if l == 0 else H
        for name, shape in (("weight_ih", (4 * H, din)), ("weight_hh", (4 * H, H)), ("bias_ih", (4 * H,)),
                            ("bias_hh", (4 * H,))):
            out[f"lstm.{name}_l{l}"] = _u(seed, stream, shape, -k, k)
            stream += 1
    kl = 1.0 / np.sqrt(H)
    out["linear.weight"] = _u(seed, stream, (E, H), -kl, kl)
    out["linear.bias"] = _u(seed, stream + 1, (E,), -kl, kl)
    return OrderedDict((n, torch.from_numpy(v).to(device)) for n, v in out.items())


def synthetic_speech(seed: int, n: int, sr: int) -> np.ndarray:
    """A deterministic speech-like test waveform in [-1, 1]: a 110-220 Hz glottal-pulse-like
    harmonic series with a slow formant sweep, syllable-rate amplitude envelope and a little
    noise, so spectra span > 80 dB like real speech."""
    t = np.arange(n, dtype=np.float64) / sr
    u = uniform01(seed, 30_000_001, 8)
    f0 = 110.0 + 110.0 * u[0] + 20.0 * np.sin(2 * np.pi * 0.7 * t)
    ph = 2 * np.pi * np.cumsum(f0) / sr
    form = 500.0 + 1500.0 * (0.5 + 0.5 * np.sin(2 * np.pi * (0.3 + u[1]) * t))
    y = np.zeros(n)
    for h in range(1, 40):
        fh = h * f0
        gain = np.exp(-((fh - form) / 400.0) ** 2) + 0.3 * np.exp(-((fh - 2.5 * form) / 600.0) ** 2) + 0.02 / h
        y += gain * np.sin(h * ph)
    env = 0.5 + 0.5 * np.sin(2 * np.pi * (3.0 + u[2]) * t) ** 2
    noise = (uniform01(seed, 30_000_003, n) - 0.5) * 2e-3
    y = y * env
    y = 0.5 * y / np.max(np.abs(y)) + noise
    return y.astype(np.float32)


# ---- WaveRNN vocoder ---------------------------------------------------

WAVERNN_DIMS = dict(rnn_dims=512, fc_dims=512, feat_dims=80, res_out_dims=128, compute_dims=128,
                    res_blocks=10, pad=2, upsample_factors=(5, 5, 11), bits=9)


def wavernn_state_dict(seed: int = 0, mode: str = "MOL", device="cpu", **dims):
    """WaveRNN.state_dict() keys/shapes (wavernn/model.py:16-180) with PyTorch's default init
    bounds (Conv/Linear U(±1/√fan_in), GRU U(±1/√H)).  BatchNorm affine and running statistics
    are drawn from small ranges (generate() runs eval-mode BN, so identities would hide bugs);
    the up-sampling smoothing kernels start at the reference's 1/k fill (model.py:85) scaled by
    U(0.8, 1.2) per tap for the same reason."""
    import torch
    d = dict(WAVERNN_DIMS)
    d.update(dims)
    R, F_, C, A, Fc = d["rnn_dims"], d["feat_dims"], d["compute_dims"], d["res_out_dims"], d["fc_dims"]
    aux = A // 4
    k_size = 2 * d["pad"] + 1
    n_classes = 2 * d["bits"] if mode == "RAW" else 30
    out = OrderedDict()
    stream = [60_000_000]

    def u(shape, lo, hi):
        v = _u(seed, stream[0], shape, lo, hi)
        stream[0] += 1
        return v

    def bn(prefix, n):
        out[prefix + ".weight"] = u((n,), 0.8, 1.2)
        out[prefix + ".bias"] = u((n,), -0.1, 0.1)
        out[prefix + ".running_mean"] = u((n,), -0.2, 0.2)
        out[prefix + ".running_var"] = u((n,), 0.5, 1.5)
        out[prefix + ".num_batches_tracked"] = np.array(0, dtype=np.int64)

    out["step"] = np.zeros(1, dtype=np.int64)
    kb = 1.0 / math.sqrt(F_ * k_size)
    out["upsample.resnet.conv_in.weight"] = u((C, F_, k_size), -kb, kb)
    bn("upsample.resnet.batch_norm", C)
    kb = 1.0 / math.sqrt(C)
    for i in range(d["res_blocks"]):
        p = f"upsample.resnet.layers.{i}"
        out[p + ".conv1.weight"] = u((C, C, 1), -kb, kb)
        out[p + ".conv2.weight"] = u((C, C, 1), -kb, kb)
        bn(p + ".batch_norm1", C)
        bn(p + ".batch_norm2", C)
    out["upsample.resnet.conv_out.weight"] = u((A, C, 1), -kb, kb)
    out["upsample.resnet.conv_out.bias"] = u((A,), -kb, kb)
    for j, s in enumerate(d["upsample_factors"]):
        k = 2 * s + 1
        out[f"upsample.up_layers.{2 * j + 1}.weight"] = (u((1, 1, 1, k), 0.8, 1.2) / k).astype(np.float32)

    def linear(name, n_out, n_in):
        kl = 1.0 / math.sqrt(n_in)
        out[name + ".weight"] = u((n_out, n_in), -kl, kl)
        out[name + ".bias"] = u((n_out,), -kl, kl)

    def gru(name, n_in):
        kg = 1.0 / math.sqrt(R)
        out[name + ".weight_ih_l0"] = u((3 * R, n_in), -kg, kg)
        out[name + ".weight_hh_l0"] = u((3 * R, R), -kg, kg)
        out[name + ".bias_ih_l0"] = u((3 * R,), -kg, kg)
        out[name + ".bias_hh_l0"] = u((3 * R,), -kg, kg)

    linear("I", R, F_ + aux + 1)
    gru("rnn1", R)
    gru("rnn2", R + aux)
    linear("fc1", Fc, R + aux)
    linear("fc2", Fc, Fc + aux)
    linear("fc3", n_classes, Fc)
    return OrderedDict((n, torch.from_numpy(np.asarray(v)).to(device)) for n, v in out.items())
