"""ORACLE — test infrastructure only (never imported by the product path).

Independent float64 numpy restatement of the Generator forward (no torch kernels at all),
used to bound the fp32 rounding of both the reference and the HIP path.  Explicit loops over
the 5 conv taps and over time; small cases only (B*T up to a few thousand frames).
References are to /root/reference/autovc/auto_encoder/*.py.
"""
from __future__ import annotations

import numpy as np

FREQ = 32


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def conv1d_k5(x, W, b):
    """Conv1d(k=5, pad=2) on channel-first x (B,Cin,T); W (Cout,Cin,5) — net_layers.py:39-42."""
    B, Cin, T = x.shape
    xp = np.zeros((B, Cin, T + 4))
    xp[:, :, 2:T + 2] = x
    y = np.zeros((B, W.shape[0], T))
    for k in range(5):
        y += np.einsum("oc,bct->bot", W[:, :, k], xp[:, :, k:k + T])
    return y + b[None, :, None]


def batchnorm(y, gamma, beta, rm, rv, training, eps=1e-5, momentum=0.1):
    """nn.BatchNorm1d over (B,T) per channel; returns (out, new_rm, new_rv)."""
    if training:
        mean = y.mean(axis=(0, 2))
        var = y.var(axis=(0, 2))
        n = y.shape[0] * y.shape[2]
        new_rm = (1 - momentum) * rm + momentum * mean
        new_rv = (1 - momentum) * rv + momentum * var * n / max(n - 1, 1)
    else:
        mean, var, new_rm, new_rv = rm, rv, rm, rv
    out = (y - mean[None, :, None]) / np.sqrt(var[None, :, None] + eps) * gamma[None, :, None] + beta[None, :, None]
    return out, new_rm, new_rv


def lstm_dir(x, Wih, Whh, bih, bhh, reverse=False):
    """One LSTM direction, gates (i,f,g,o), zero initial state. x (B,T,D) -> (B,T,H)."""
    B, T, _ = x.shape
    H = Whh.shape[1]
    h = np.zeros((B, H))
    c = np.zeros((B, H))
    out = np.zeros((B, T, H))
    gx = x @ Wih.T + bih + bhh
    order = range(T - 1, -1, -1) if reverse else range(T)
    for t in order:
        g = gx[:, t] + h @ Whh.T
        i, f, gg, o = _sig(g[:, :H]), _sig(g[:, H:2 * H]), np.tanh(g[:, 2 * H:3 * H]), _sig(g[:, 3 * H:])
        c = f * c + i * gg
        h = o * np.tanh(c)
        out[:, t] = h
    return out


def lstm(x, sd, prefix, layers, bidir):
    for l in range(layers):
        outs = []
        for sfx in ([""] + (["_reverse"] if bidir else [])):
            p = [sd[f"{prefix}.{n}_l{l}{sfx}"] for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
            outs.append(lstm_dir(x, *p, reverse=(sfx == "_reverse")))
        x = np.concatenate(outs, axis=-1)
    return x


def forward(sd, x, c_org, c_trg, training=True):
    """AutoEncoder.forward (model.py:68-146) in float64. Returns (mel, mel_post, codes, new_bn)."""
    sd = {k: np.asarray(v, dtype=np.float64) for k, v in sd.items()}
    x = np.asarray(x, np.float64)
    B, _, T = x.shape
    new_bn = {}

    def cbn(h, prefix):
        y = conv1d_k5(h, sd[prefix + ".0.conv.weight"], sd[prefix + ".0.conv.bias"])
        out, rm, rv = batchnorm(y, sd[prefix + ".1.weight"], sd[prefix + ".1.bias"],
                                sd[prefix + ".1.running_mean"], sd[prefix + ".1.running_var"], training)
        new_bn[prefix + ".1.running_mean"] = rm
        new_bn[prefix + ".1.running_var"] = rv
        return out

    h = np.concatenate([x, np.repeat(np.asarray(c_org, np.float64)[:, :, None], T, axis=2)], axis=1)
    for i in range(3):
        h = np.maximum(cbn(h, f"encoder.convolutions.{i}"), 0.0)
    out = lstm(h.transpose(0, 2, 1), sd, "encoder.lstm", 2, True)
    fwd, bwd = out[:, :, :32], out[:, :, 32:]
    ca = [fwd[:, i] for i in range(FREQ - 1, T, FREQ)]
    cb = [bwd[:, i] for i in range(0, T, FREQ)]
    codes = np.concatenate(ca + cb, axis=-1)
    if c_trg is None:
        return codes
    up = np.zeros((B, 64, T))
    for t in range(T):
        up[:, :32, t] = ca[min(t // FREQ, len(ca) - 1)]
        up[:, 32:, t] = cb[t // FREQ]
    enc = np.concatenate([up, np.repeat(np.asarray(c_trg, np.float64)[:, :, None], T, axis=2)], axis=1)
    h = lstm(enc.transpose(0, 2, 1), sd, "decoder.lstm1", 1, False).transpose(0, 2, 1)
    for i in range(3):
        h = np.maximum(cbn(h, f"decoder.convolutions.{i}"), 0.0)
    out = lstm(h.transpose(0, 2, 1), sd, "decoder.lstm2", 2, False)
    mel = (out @ sd["decoder.linear_projection.linear_layer.weight"].T
           + sd["decoder.linear_projection.linear_layer.bias"]).transpose(0, 2, 1)
    p = mel
    for i in range(4):
        p = np.tanh(cbn(p, f"postnet.convolutions.{i}"))
    p = cbn(p, "postnet.convolutions.4")
    return mel, mel + p, codes, new_bn
