"""Timing experiments on the persistent BPTT (avc_debug_bptt_diag; results are not valid while a
bit is set): 1 = no dG operand loads in the product phase, 2 = no partial loads in the epilogue
phase, 4 = no waits between the phases, 8 = no partial stores in the product phase, 16 = no dG / dc
stores in the epilogue phase, 32 = no drains before the counter adds."""
import sys

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
    for bits in [int(b) for b in sys.argv[1:]] or (0, 1, 2, 4, 3, 7):
        _lib.call("avc_debug_bptt_diag", bits)
        for rep in range(3):
            y = ops.LSTMLayer.apply(x, *ws, T, B, True)
            torch.cuda.synchronize()
            if rep == 2:
                _lib.timing_enable(["lstm_step_bwd"])
                _lib.timing_reset()
            y.backward(dy)
            torch.cuda.synchronize()
            x.grad = None
            for w in ws:
                w.grad = None
        r = _lib.timing_read("lstm_step_bwd")
        _lib.timing_enable([])
        print(f"H={H} diag={bits}: {1e3 * r['ms'] / T:.1f} us per step", flush=True)
_lib.call("avc_debug_bptt_diag", 0)
