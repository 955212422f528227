"""Diagnostic: the C2 forward GEMM shapes timed on the normal library and on a build whose
gemm16f skips its global->LDS DMA (-DAVC_GEMM_NOLOAD=1, diag/libautovc_hip_noload.so; the MFMAs
run on stale LDS).  The difference is the time the kernel spends waiting for operands.
    AUTOVC_HIP_LIB=diag/libautovc_hip_noload.so python scripts/gemm_noload.py"""
import os
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
T, B = 128, 64
M = T * B
g = torch.Generator(device="cpu").manual_seed(3)
x = torch.rand(M, 512, generator=g).to(dev)
W = ((torch.rand(512, 512, 5, generator=g) - 0.5) * 0.1).to(dev)
bz = torch.zeros(512, device=dev)
on = torch.ones(512, device=dev)
a = torch.rand(M, 512, generator=g).to(dev)
w2 = (torch.rand(4096, 512, generator=g) * 0.05).to(dev)
_lib.timing_enable(["gemm"])


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    _lib.timing_reset()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    r = _lib.timing_read("gemm")
    return 1000 * r["ms"] / r["launches"], r["flops"] / r["launches"]


with torch.no_grad():
    tc, fc = timed(lambda: ops.ConvBNAct.apply(x, W, bz, on, bz, None, None, True, 0.1, 1e-5, 1, None, T, B))
    tl, fl = timed(lambda: ops.Linear.apply(a, w2, None))
lib = os.path.basename(os.environ.get("AUTOVC_HIP_LIB", "libautovc_hip.so"))
print(f"{lib}: conv 512->512 k5 GEMM {tc:.1f} us ({fc / tc / 1e6:.0f} TFLOP/s), "
      f"lstm2 input projection {tl:.1f} us ({fl / tl / 1e6:.0f} TFLOP/s)", flush=True)
