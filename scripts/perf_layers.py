"""Per-layer timing on the GPU (HIP events around each op call): conv+BN, LSTM layers, GEMM."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    cfgs = [int(c) for c in sys.argv[1:]] or [0]
    for c in cfgs:
        _lib.call("avc_gemm_config", c)
        run(f"cfg{c}")
    _lib.call("avc_gemm_config", 8)


def run(tag):
    dev = torch.device("cuda:0")
    B, T = 64, 128
    M = B * T
    out = {}
    with torch.no_grad():
        for cin, cout in [(336, 512), (512, 512), (80, 512), (512, 80)]:
            x = torch.rand(M, cin, device=dev)
            W = (torch.rand(cout, cin, 5, device=dev) - 0.5) * 0.1
            b = torch.zeros(cout, device=dev)
            g = torch.ones(cout, device=dev)
            ms = timeit(lambda: ops.ConvBNAct.apply(x, W, b, g, b, None, None, True, 0.1, 1e-5, 1, None, T, B))
            fl = 2.0 * M * cout * cin * 5
            out[f"conv_bn {cin}->{cout}"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
        for din, H in [(320, 512), (512, 1024), (1024, 1024), (512, 32)]:
            x = torch.rand(M, din, device=dev)
            k = 1.0 / H ** 0.5
            wi = (torch.rand(4 * H, din, device=dev) * 2 - 1) * k
            wh = (torch.rand(4 * H, H, device=dev) * 2 - 1) * k
            bi = torch.zeros(4 * H, device=dev)
            ms = timeit(lambda: ops.LSTMLayer.apply(x, wi, wh, bi, bi, T, B, False), reps=3, warm=1)
            fl = 2.0 * M * 4 * H * (din + H)
            out[f"lstm {din}->{H}"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
                                       "us_per_step": round(1000 * ms / T, 2)}
        for (m, n, kk) in [(8192, 4096, 1024), (8192, 512, 2560), (4096, 1024, 8192)]:
            a = torch.rand(m, kk, device=dev)
            bb = torch.rand(kk, n, device=dev)
            ms = timeit(lambda: ops.gemm(a, bb))
            out[f"gemm {m}x{n}x{kk}"] = {"ms": round(ms, 4), "tflops": round(2.0 * m * n * kk / ms / 1e9, 1)}
    print(tag, json.dumps({k: v["ms"] for k, v in out.items()}))


if __name__ == "__main__":
    main()
