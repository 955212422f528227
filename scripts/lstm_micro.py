"""Microbenchmark: the decoder.lstm2 pair (pipelined) and single layers at C2 size, for PMC runs."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
T, B, H = 128, 64, 1024
k = 1.0 / H ** 0.5
x = torch.rand(T * B, 1024, device=dev)
wi = (torch.rand(4 * H, 1024, device=dev) * 2 - 1) * k
wh = (torch.rand(4 * H, H, device=dev) * 2 - 1) * k
bi = torch.zeros(4 * H, device=dev)
with torch.no_grad():
    for _ in range(3):
        ops.LSTMLayer.apply(x, wi, wh, bi, bi, T, B, False)
torch.cuda.synchronize()
print("done")
