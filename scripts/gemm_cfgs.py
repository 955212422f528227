"""gemm16f variants (avc_gemm_config) on the C2 GEMM shapes: 512->512 conv+BN forward (M = 8192,
K = 5 x 512) and the lstm2 input projection (8192 x 4096 x 512), plus the whole fused C2 forward.
Checks every variant is bit-identical to the default (the arithmetic is the same)."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

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
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
xm = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)


def timed(fn, reps=20):
    for _ in range(3):
        out = fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6, out


ref = None
cfgs = [int(v) for v in sys.argv[1:]] or [1, 2, 3, 4, 5, 1]
with torch.no_grad():
    for cfg in cfgs:
        _lib.call("avc_gemm_config", cfg)
        tc, oc = timed(lambda: ops.ConvBNAct.apply(x, W, bz, on, bz, None, None, True, 0.1, 1e-5, 1, None, T, B))
        tl, ol = timed(lambda: ops.Linear.apply(a, w2, None))
        tf, of = timed(lambda: ae(xm, co, ct))
        outs = [oc.clone(), ol.clone()] + [o.clone() for o in of]
        if ref is None:
            ref = outs
        same = all(torch.equal(p, q) for p, q in zip(outs, ref))
        print(f"cfg {cfg:2d}: conv+BN {tc:7.1f} us  lstm2-proj {tl:7.1f} us  C2 forward {tf / 1e3:6.3f} ms  "
              f"bit-identical {same}", flush=True)
_lib.call("avc_gemm_config", 8)
