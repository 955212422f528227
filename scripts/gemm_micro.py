"""Microbenchmark for PMC runs of the split-f16 GEMM (gemm16f_kernel), 5 reps of each shape:
  * C2: the 512->512 conv+BN forward at B = 64 (M = 8192, K = 2560) and the lstm2 input
    projection (8192 x 4096 x 512) as a Linear;
  * C3 (B = 256, M = 32768): the 512->512 conv+BN forward, then its backward (dgrad: dX = dY Wd,
    K = 2560; wgrad: dW = dY^T X per tap, K = M) through the training autograd path."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
which = sys.argv[1] if len(sys.argv) > 1 else "all"


def conv(T, B, backward):
    """5 forwards, or (backward) ONE forward and 5 backwards of it (so the C3 dgrad, whose grid
    equals the forward's, dominates that grid's counter averages)."""
    M = T * B
    x = torch.rand(M, 512, device=dev, requires_grad=backward)
    W = ((torch.rand(512, 512, 5, device=dev) - 0.5) * 0.1).requires_grad_(backward)
    b = torch.zeros(512, device=dev, requires_grad=backward)
    g = torch.ones(512, device=dev, requires_grad=backward)
    bt = torch.zeros(512, device=dev, requires_grad=backward)
    d = torch.rand(M, 512, device=dev) - 0.5
    with torch.set_grad_enabled(backward):
        for _ in range(1 if backward else 5):
            y = ops.ConvBNAct.apply(x, W, b, g, bt, None, None, True, 0.1, 1e-5, 1, None, T, B)
    if backward:
        for _ in range(5):
            y.backward(d, retain_graph=True)


if which in ("all", "c2"):
    conv(128, 64, False)
    a = torch.rand(8192, 512, device=dev)
    w2 = torch.rand(4096, 512, device=dev) * 0.05
    with torch.no_grad():
        for _ in range(5):
            ops.Linear.apply(a, w2, None)
if which in ("all", "c3fwd"):
    conv(128, 256, False)
if which in ("all", "c3bwd"):
    conv(128, 256, True)
torch.cuda.synchronize()
print("done")
