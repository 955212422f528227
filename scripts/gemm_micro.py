"""Microbenchmark for PMC runs: the C2 512->512 conv+BN forward (gemm16 path) and the LSTM2
input projection (8192 x 4096 x 512), 5 reps each."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
T, B = 128, 64
M = T * B
x = torch.rand(M, 512, device=dev)
W = (torch.rand(512, 512, 5, device=dev) - 0.5) * 0.1
b = torch.zeros(512, device=dev)
g = torch.ones(512, device=dev)
a = torch.rand(M, 512, device=dev)
w2 = torch.rand(4096, 512, device=dev) * 0.05
with torch.no_grad():
    for _ in range(5):
        ops.ConvBNAct.apply(x, W, b, g, b, None, None, True, 0.1, 1e-5, 1, None, T, B)
    for _ in range(5):
        ops.Linear.apply(a, w2, None)
torch.cuda.synchronize()
print("done")
