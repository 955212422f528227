"""A/B of the XCD-local BPTT (avc_bptt_xcd values in argv, default 0 1) on C3's lstm1 backward
(B = 256, T = 128, din = 320, H = 512), alternating in one process: median ms per LSTMLayer
backward (the BPTT plus its weight-gradient / dX products), and bit-identity of every gradient
against the first value."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402

B, T, din, H = 256, 128, 320, 512
vals = [int(v) for v in sys.argv[1:]] or [0, 1]
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(3)
k = 1.0 / H ** 0.5
ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev).requires_grad_(True)
      for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
x = (torch.randn(T * B, din, generator=g) * 0.5).to(dev).requires_grad_(True)
dy = torch.randn(T * B, H, generator=g).to(dev)


def setv(v):
    _lib.call("avc_bptt_xcd", v)


def run():
    for p in ws + [x]:
        p.grad = None
    y = ops.LSTMLayer.apply(x, *ws, T, B, True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    y.backward(dy)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, [x.grad.clone()] + [w.grad.clone() for w in ws]


res = {v: [] for v in vals}
ref = None
same = {v: True for v in vals}
for rep in range(6):
    for v in vals:
        setv(v)
        run()
        ms, grads = run()
        res[v].append(ms)
        if ref is None:
            ref = grads
        same[v] &= all(torch.equal(a, b) for a, b in zip(grads, ref))
setv(1)
for v in vals:
    print(f"flags {v}: backward median {np.median(res[v]):.3f} ms ({', '.join(f'{t:.3f}' for t in res[v])}); "
          f"bit-identical {same[v]}", flush=True)
