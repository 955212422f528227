"""Sweep Linear shapes on the pre-split fragment GEMM (mode 2) vs mode 1; print max errors."""
import itertools
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
for M, K, N in itertools.product([64, 128, 256, 1024], [64, 128, 256, 512], [32, 128]):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(M, K, generator=g).to(dev)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
    out = {}
    for mode in (1, 2):
        _lib.call("avc_gemm_tune", mode)
        with torch.no_grad():
            out[mode] = ops.Linear.apply(x, w, None)
    torch.cuda.synchronize()
    d = (out[1] - out[2]).abs()
    bad = (d > 1e-4).nonzero()
    info = ""
    if len(bad):
        rows = sorted(set(bad[:, 0].tolist()))
        cols = sorted(set(bad[:, 1].tolist()))
        info = f" bad rows {rows[:6]}..({len(rows)}) cols {cols[:6]}..({len(cols)})"
    print(f"M={M:5d} K={K:4d} N={N:4d} maxdiff {d.max().item():.3e}{info}", flush=True)
_lib.call("avc_gemm_tune", 2)
