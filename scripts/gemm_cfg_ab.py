"""A/B of gemm16f tile/ring configurations (avc_gemm_config) in one process, alternating: the C2
512->512 conv+BN forward, the lstm2 input projection, and a C3 (B=256) conv+BN forward + backward
(dgrad + wgrad); per-config kernel time from the library's GEMM timing events and a bit-identity
check of every output against the first configuration."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
cfgs = [int(c) for c in sys.argv[1:]] or [8, 1, 8, 1, 8, 1]
g = torch.Generator(device="cpu").manual_seed(5)


def rnd(*shape, scale=1.0):
    return ((torch.rand(*shape, generator=g) - 0.5) * scale).to(dev)


def conv_case(T, B, backward):
    M = T * B
    x = rnd(M, 512).requires_grad_(backward)
    W = rnd(512, 512, 5, scale=0.1).requires_grad_(backward)
    z = torch.zeros(512, device=dev, requires_grad=backward)
    o = torch.ones(512, device=dev, requires_grad=backward)
    d = rnd(M, 512)

    def run():
        with torch.set_grad_enabled(backward):
            y = ops.ConvBNAct.apply(x, W, z, o, z, None, None, True, 0.1, 1e-5, 1, None, T, B)
            if not backward:
                return [y]
            gx, gw = torch.autograd.grad(y, (x, W), d)
            return [y, gx, gw]
    return run


a = rnd(8192, 512)
w2 = rnd(4096, 512, scale=0.1)
cases = {"c2 conv": conv_case(128, 64, False), "lstm2 inproj": lambda: [ops.Linear.apply(a, w2, None)],
         "c3 conv fwd+bwd": conv_case(128, 256, True)}
ref = {}
_lib.timing_enable(["gemm"])
for cfg in cfgs:
    _lib.call("avc_gemm_config", cfg)
    line = []
    for name, fn in cases.items():
        with torch.no_grad() if name != "c3 conv fwd+bwd" else torch.enable_grad():
            for _ in range(2):
                out = fn()
            torch.cuda.synchronize()
            _lib.timing_reset()
            for _ in range(10):
                out = fn()
            torch.cuda.synchronize()
        r = _lib.timing_read("gemm")
        us = 1e3 * r["ms"] / r["launches"]
        tf = r["flops"] / (r["ms"] * 1e-3) / 1e12
        out = [o.detach().clone() for o in out]
        same = name not in ref or all(torch.equal(u, v) for u, v in zip(out, ref[name]))
        ref.setdefault(name, out)
        err = ""
        if name == "lstm2 inproj":  # accuracy of the plain product against float64
            err = f", max|d| vs f64 {float((out[0].double() - a.double() @ w2.double().T).abs().max()):.2e}"
        line.append(f"{name} {us:.1f} us/launch ({tf:.0f} TF/s){err}{'' if same else ' NOT bit-identical'}")
    print(f"cfg {cfg}: " + "; ".join(line), flush=True)
_lib.call("avc_gemm_config", 8)
