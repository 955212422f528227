"""A/B of the persistent recurrences' input slot (avc_lstm_persist_inproj) and hand-off form
(avc_lstm_persist_tune 1 / 2) inside the fused C2 forward: per-launch time of the lstm2 / lstm1
persistent classes and of the GEMM class, and the wall time per forward (graph replay)."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
B, T = (int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (64, 128)))
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(5, B, T)).to(dev)
co = torch.from_numpy(synthetic_embedding(6, B)).to(dev)
classes = ["lstm2_persist", "lstm1_persist", "gemm"]
for rep in range(2):
    for mode, inproj in ((2, 0), (2, 1), (2, 2), (2, 3)):
        _lib.call("avc_lstm_persist_tune", mode)
        _lib.call("avc_lstm_persist_inproj", inproj)
        with torch.no_grad():
            for _ in range(3):
                ae(x, co, co)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                ae(x, co, co)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / 20 * 1e3
            _lib.timing_enable(classes)
            _lib.timing_reset()
            for _ in range(5):
                ae(x, co, co)
            torch.cuda.synchronize()
            r = {c: _lib.timing_read(c) for c in classes}
            _lib.timing_enable([])
        per = "  ".join(f"{c} {1e3 * r[c]['ms'] / max(r[c]['launches'], 1):7.1f} us x{r[c]['launches'] // 5}"
                        for c in classes)
        print(f"mode {mode} inproj {inproj}: {wall:.3f} ms/forward  {per}", flush=True)
_lib.call("avc_lstm_persist_tune", 2)
_lib.call("avc_lstm_persist_inproj", 1)
