"""Fused C2 forward (B=64, T=128) under each decoder.lstm2 path: 0 = T+2 step launches
(lstm_split.hip), 1 = weight-stationary launch with acquire hand-offs, 2 = with sc1-load
hand-offs; an argument "m:d" also sets the split-h prefetch depth d (avc_lstm_persist_depth).
Prints ms per forward (graph replay, 20 reps) and checks outputs are bit-identical."""
import ctypes
import sys
import time

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
B, T = 64, 128
modes = sys.argv[1:] or ["0", "1", "2", "1", "2"]
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
ref = None
for spec in modes:
    mode, _, depth = spec.partition(":")
    mode = int(mode)
    _lib.call("avc_lstm_persist_tune", mode)
    _lib.call("avc_lstm_persist_depth", int(depth or 2))
    with torch.no_grad():
        for _ in range(3):
            out = ae(x, co, ct)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            out = ae(x, co, ct)
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    if ref is None:
        ref = [o.clone() for o in out]
    same = all(torch.equal(a, b) for a, b in zip(out, ref))
    dmax = max((a - b).abs().max().item() for a, b in zip(out, ref))
    print(f"mode {spec}: {ms:.3f} ms per forward, {B * T / ms * 1e3 / 1e6:.3f} M frames/s, bit-identical {same} "
          f"(max|d| {dmax:.2e})")
g = ctypes.c_long(0)
_lib.call("avc_lstm_persist_status", ctypes.byref(g))
print("giveups", g.value)
_lib.call("avc_lstm_persist_tune", 2)
_lib.call("avc_lstm_persist_depth", 2)
