"""A/B of the BPTT recurrence modes (avc_bptt_mode, avc_bptt_persist) at the C3 layer shapes: one LSTM layer
forward + backward at B = 256, T = 128 (H = 1024 / din = 1024 like decoder.lstm2's layer 1,
H = 512 / din = 320 like decoder.lstm1); prints the backward time per call and the per-step
BPTT kernel times from the library's timing class."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
B, T = 256, 128
# a mode: "<avc_bptt_mode>:<avc_bptt_persist>" (e.g. 1:1 persistent, 1:0 launch per step)
modes = [tuple(int(x) for x in v.split(":")) for v in sys.argv[1:]] or [(1, 1), (1, 0), (0, 0)]
for H, din in ((1024, 1024), (512, 320)):
    g = torch.Generator().manual_seed(H)
    k = 1.0 / H ** 0.5
    ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev).requires_grad_(True)
          for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    x = (torch.randn(T * B, din, generator=g) * 0.5).to(dev).requires_grad_(True)
    dy = torch.randn(T * B, H, generator=g).to(dev)
    for mode in modes:
        _lib.call("avc_bptt_mode", mode[0])
        _lib.call("avc_bptt_persist", mode[1])
        ts = []
        for rep in range(6):
            y = ops.LSTMLayer.apply(x, *ws, T, B, True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            y.backward(dy)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            x.grad = None
            for w in ws:
                w.grad = None
        ts.sort()
        print(f"H={H} din={din} mode {mode}: backward {1e3 * ts[len(ts) // 2]:.2f} ms", flush=True)
_lib.call("avc_bptt_mode", 1)
_lib.call("avc_bptt_persist", 1)
