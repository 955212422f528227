"""Whole-Generator mel_post error (B = 1, T = 128, seeds 0-2) when decoder.lstm2's products are
emulated in other number formats, everything else in float64, against the float64 oracle; the
fp32 reference's own distance is printed beside it.  Formats: 3xf16 (the kernels'
hi.hi + hi.lo + lo.hi of per-row-scaled W and h * 2^15), and int8 limbs (W per row and h as 23-bit
fixed point in three balanced 8-bit limbs, the products of limb pairs with i + j <= 2 -- 6
v_mfma_i32_16x16x64_i8 products, the 3xf16 MFMA cost at 3 bytes per h element -- or <= 3, 8
products).  CPU only; uses the oracle as the checker."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import autovc_oracle as orc
from autovc_amd.weights import torch_state_dict, synthetic_mel, synthetic_embedding
torch.set_num_threads(8)

def limbs(V):
    L2 = ((V + 128) % 256) - 128
    V1 = (V - L2) // 256
    L1 = ((V1 + 128) % 256) - 128
    L0 = (V1 - L1) // 256
    return L0, L1, L2

def q_rows(W, bits=22):   # W [N][K] per-row power-of-two -> integer limbs
    e = np.floor(np.log2(np.abs(W).max(1) + 1e-300)) + 1
    s = 2.0 ** (bits - e)
    return limbs(np.rint(W * s[:, None]).astype(np.int64)), s

def prod_i8(h, Wq, nprod):
    (w0, w1, w2), sw = Wq
    sh = 2.0 ** 22
    h0, h1, h2 = limbs(np.rint(h * sh).astype(np.int64))
    m = lambda a, b: (a @ b.T).astype(np.float64)
    acc = m(h0, w0) * 2.0**32 + (m(h0, w1) + m(h1, w0)) * 2.0**24 + (m(h0, w2) + m(h1, w1) + m(h2, w0)) * 2.0**16
    if nprod >= 8:
        acc += (m(h1, w2) + m(h2, w1)) * 2.0**8
    return acc / (sw[None, :] * sh)

def prod_3f16(h, W):
    e = np.floor(np.log2(np.abs(W).max(1) + 1e-300)) + 1
    s = 2.0 ** (15 - e)[:, None]
    def split(a, sc):
        v = a * sc; hi = v.astype(np.float16).astype(np.float64); lo = (v - hi).astype(np.float16).astype(np.float64)
        return hi / sc, lo / sc
    wh, wl = split(W, s); hh, hl = split(h, 2.0 ** 15)
    return hh @ wh.T + hh @ wl.T + hl @ wh.T

MODE = None
def lstm_emu(x, sd, prefix, num_layers, bidirectional):
    if prefix != "decoder.lstm2" or MODE is None:
        return ORIG(x, sd, prefix, num_layers, bidirectional)
    xs = x.double().numpy()          # [B][T][D]
    B, T, _ = xs.shape
    inp = xs
    for L in range(num_layers):
        Wih = sd[f"{prefix}.weight_ih_l{L}"].double().numpy(); Whh = sd[f"{prefix}.weight_hh_l{L}"].double().numpy()
        b = (sd[f"{prefix}.bias_ih_l{L}"] + sd[f"{prefix}.bias_hh_l{L}"]).double().numpy()
        H = Whh.shape[1]
        if MODE[0] == "i8":
            qih, qhh = q_rows(Wih), q_rows(Whh)
            P = (lambda a, W, q: prod_i8(a, q, MODE[1]))
        else:
            qih = qhh = None
            P = (lambda a, W, q: prod_3f16(a, W))
        h = np.zeros((B, H)); c = np.zeros((B, H)); out = np.zeros((B, T, H))
        # layer 0's input projection on the GPU is a 3xf16 product (input slot); layer 1's is slot 1
        gx = [ (inp[:, t] @ Wih.T if L == 0 else P(inp[:, t], Wih, qih)) + b for t in range(T)]
        for t in range(T):
            g = gx[t] + (P(h, Whh, qhh) if t > 0 else 0.0)
            i, f, gg, o = np.split(g, 4, axis=1)
            sg = lambda z: 1 / (1 + np.exp(-z))
            c = sg(f) * c + sg(i) * np.tanh(gg); h = sg(o) * np.tanh(c); out[:, t] = h
        inp = out
    return torch.from_numpy(inp).to(x.dtype)

ORIG = orc.lstm
orc.lstm = lstm_emu
for seed in (0, 1, 2):
    for B, T in ((1, 128),):
        sd = torch_state_dict(seed)
        x = synthetic_mel(5 + seed, B, T); co = synthetic_embedding(101, B); ct = synthetic_embedding(201, B)
        def run(dtype, mode):
            global MODE
            MODE = mode
            s = {k: (v.to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
            bufs = {k: v for k, v in s.items() if "running" in k or "num_batches" in k}
            with torch.no_grad():
                return orc.forward(s, *(torch.from_numpy(a).to(dtype) for a in (x, co, ct)), True, bufs)[1].double()
        e64 = run(torch.float64, None); r32 = run(torch.float32, None)
        res = {"ref32": float((r32 - e64).abs().max())}
        for m in (("f16",), ("i8", 6), ("i8", 8)):
            v = run(torch.float64, m)
            res[m[0] + (str(m[1]) if len(m) > 1 else "")] = float((v - e64).abs().max())
        print(f"seed {seed} B={B} T={T}: mel_post vs f64: " + ", ".join(f"{k} {v:.2e}" for k, v in res.items()), flush=True)
