"""Sweep the split-fp16 LSTM step's K range per workgroup at C2 size (whole Generator forward,
plus the decoder lstm1 / single H=1024 layers alone)."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
B, T = 64, 128
model = AutoEncoder(device=dev, verbose=False)
model.load_state_dict(torch_state_dict(0))
model.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
c1 = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
c2 = torch.from_numpy(synthetic_embedding(201, B)).to(dev)


def layer(din, H):
    k = 1.0 / H ** 0.5
    xi = torch.rand(T * B, din, device=dev)
    wi = (torch.rand(4 * H, din, device=dev) * 2 - 1) * k
    wh = (torch.rand(4 * H, H, device=dev) * 2 - 1) * k
    bi = torch.zeros(4 * H, device=dev)
    return lambda: ops.LSTMLayer.apply(xi, wi, wh, bi, bi, T, B, False)


cases = {"generator": lambda: model(x, c1, c2), "lstm H=512": layer(320, 512), "lstm H=1024": layer(1024, 1024)}
for ks, nc, r64 in [(0, 0, 0), (0, 0, 1), (0, 4, 0), (1024, 4, 0)]:
    _lib.call("avc_lstm_split_tune", ks, nc, r64)
    row = {}
    for name, fn in cases.items():
        with torch.no_grad():
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 5 * 1000
            _lib.timing_enable(["lstm_step_fwd"])
            _lib.timing_reset()
            fn()
            torch.cuda.synchronize()
            r = _lib.timing_read("lstm_step_fwd")
            _lib.timing_enable([])
        row[name] = {"ms": round(ms, 3), "step_us": round(1000 * r["ms"] / max(1, r["launches"]), 2),
                     "launches": r["launches"]}
    print(f"kslice={ks} nc={nc} rows64={r64}", json.dumps(row), flush=True)
_lib.call("avc_lstm_split_tune", 0, 0, 0)
