"""Probe: does a persistent BPTT launch dispatched beside a CU-holding kernel give up?
Times the hog alone, then hog + one persistent lstm2-layer backward (B=256, H=1024)."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autovc_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
ctx = _lib.context(dev)
hs = torch.cuda.Stream(device=dev)
n_wg = int(sys.argv[1]) if len(sys.argv) > 1 else 64
spin = int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 14)


def giveups():
    n = ctypes.c_long(0)
    _lib.call("avc_lstm_persist_status", ctypes.byref(n))
    return n.value


def hog(us):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(hs)
    _lib.call("avc_debug_hog", ctx, n_wg, 160 * 1024, us, hs.cuda_stream)
    e1.record(hs)
    n, t0 = ctypes.c_int(0), time.time()
    while n.value < n_wg and time.time() - t0 < 20:
        _lib.call("avc_debug_hog_resident", ctx, ctypes.byref(n))
    print(f"hog resident {n.value}/{n_wg} after {1e3 * (time.time() - t0):.2f} ms", flush=True)
    return e0, e1


e0, e1 = hog(100_000)
torch.cuda.synchronize()
print(f"hog alone: {e0.elapsed_time(e1):.1f} ms (asked 100 ms)", flush=True)

T, B, H = 64, 256, 1024
x = torch.randn(T * B, H, device=dev)
w_ih = torch.randn(4 * H, H, device=dev) * 0.03
w_hh = torch.randn(4 * H, H, device=dev) * 0.03
b = torch.zeros(4 * H, device=dev)
for p in (w_ih, w_hh):
    p.requires_grad_(True)
def run(label, with_hog):
    y = ops.LSTMLayer.apply(x, w_ih, w_hh, b, b, T, B, True)
    torch.cuda.synchronize()
    g0 = giveups()
    n0 = _lib.persist_launches(dev)
    if with_hog:
        h0, h1 = hog(300_000)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.time()
    s0.record()
    y.backward(torch.ones_like(y))
    s1.record()
    torch.cuda.synchronize()
    extra = f", hog {h0.elapsed_time(h1):.1f} ms, hog start -> bwd start {h0.elapsed_time(s0):.1f} ms" if with_hog else ""
    print(f"{label}: wall {1e3 * (time.time() - t0):.1f} ms, stream span {s0.elapsed_time(s1):.2f} ms, persistent "
          f"launches {_lib.persist_launches(dev) - n0}, giveups {giveups() - g0}{extra}", flush=True)


print("eligible", _lib.load().avc_bptt_persist_eligible(T, B, H), flush=True)
_lib.call("avc_debug_persist_spin_limit", spin)
run("warm-up, no hog", False)
run("no hog", False)
run("beside hog", True)
_lib.call("avc_debug_persist_spin_limit", 0)
try:
    _lib.call("avc_persist_check", ctx, torch.cuda.current_stream(dev).cuda_stream, None)
    print("health ok")
except RuntimeError as e:
    print("health:", e)
