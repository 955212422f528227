"""A/B of the persistent BPTT's epilogue mapping (avc_bptt_coalesce 0 / 1), alternating in one
process: per-launch time of the recurrence (timing class lstm_step_bwd) at B = 256, T = 128 for
H = 1024 and H = 512 (decoder lstm2 / lstm1 shapes)."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
B, T = 256, 128
for H, din in ((1024, 1024), (512, 320)):
    g = torch.Generator().manual_seed(H)
    k = 1.0 / H ** 0.5
    ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev).requires_grad_(True)
          for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    x = (torch.randn(T * B, din, generator=g) * 0.5).to(dev).requires_grad_(True)
    dy = torch.randn(T * B, H, generator=g).to(dev)
    res = {0: [], 1: []}
    for rep in range(6):
        for mode in (0, 1):
            _lib.call("avc_bptt_coalesce", mode)
            y = ops.LSTMLayer.apply(x, *ws, T, B, True)
            torch.cuda.synchronize()
            _lib.timing_enable(["lstm_step_bwd"])
            _lib.timing_reset()
            y.backward(dy)
            torch.cuda.synchronize()
            r = _lib.timing_read("lstm_step_bwd")
            _lib.timing_enable([])
            res[mode].append(1e3 * r["ms"] / max(1, r["launches"]))
            x.grad = None
            for w in ws:
                w.grad = None
    for mode in (0, 1):
        v = res[mode][1:]
        print(f"H={H} coalesce={mode}: BPTT launch median {np.median(v):.1f} us ({', '.join(f'{t:.0f}' for t in v)})",
              flush=True)
_lib.call("avc_bptt_coalesce", 1)
