"""Timing experiment: the encoder BiLSTM forward (H = 32) at C2 (B=64, T=128) and C5 (B=32, T=1024)
shapes under avc_lstm32_tune 4 (one wave), 1 (memory wave, the default), 2 (no output stores), 3 (no stores,
no input loads);
modes 2 / 3 give invalid outputs and exist only to price the step's memory operations."""
import sys
sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402
from autovc_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
for B, T in ((64, 128), (32, 1024)):
    g = torch.Generator().manual_seed(1)
    H, din = 32, 512
    ws = [(torch.rand(*s, generator=g) * 0.2 - 0.1).to(dev) for s in [(128, din), (128, H), (128,), (128,)] * 2]
    x = torch.randn(T * B, din, generator=g).to(dev)
    for mode in (4, 2, 3, 1, 4, 1):
        _lib.call("avc_lstm32_tune", mode)
        with torch.no_grad():
            for _ in range(3):
                ops.BiLSTMLayer.apply(x, *ws, T, B, False)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.BiLSTMLayer.apply(x, *ws, T, B, False)
            e1.record()
            torch.cuda.synchronize()
        print(f"B={B} T={T} mode {mode}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per BiLSTM layer "
              f"(input projection + recurrence)", flush=True)
_lib.call("avc_lstm32_tune", 1)
