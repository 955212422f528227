"""A/B of one persistent-recurrence tuning hook (argv[1], e.g. avc_lstm_persist_qwait; values argv[2:]): fused forward at C2
(B=64, T=128) and at a C5-like shape (B=32, T=1024), alternating 0 / 1 in one process; ms per
forward (graph replay, 20 reps), per-kernel times from the library's timing events, and a
bit-identity check of the outputs against the first run."""
import ctypes
import sys
import time

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
hook = sys.argv[1]
seq = [int(v) for v in sys.argv[2:]] or [0, 1, 0, 1, 0, 1]
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
for B, T in ((64, 128), (32, 1024)):
    x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
    co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
    ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
    ref = None
    for q in seq:
        _lib.call(hook, q)
        with torch.no_grad():
            for _ in range(3):
                out = ae(x, co, ct)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                out = ae(x, co, ct)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 20 * 1e3
            _lib.timing_enable(["lstm2_persist", "lstm1_persist"])
            _lib.timing_reset()
            for _ in range(5):
                ae(x, co, ct)
            torch.cuda.synchronize()
            k2, k1 = _lib.timing_read("lstm2_persist"), _lib.timing_read("lstm1_persist")
            _lib.timing_enable([])
        if ref is None:
            ref = [o.clone() for o in out]
        same = all(torch.equal(a, b) for a, b in zip(out, ref))
        print(f"B={B} T={T} {hook} {q}: {ms:.3f} ms per forward; lstm2 {1e3 * k2['ms'] / max(1, k2['launches']):.1f} us, "
              f"lstm1 {1e3 * k1['ms'] / max(1, k1['launches']):.1f} us per launch; bit-identical {same}", flush=True)
g = ctypes.c_long(0)
_lib.call("avc_lstm_persist_status", ctypes.byref(g))
print("giveups", g.value)
_lib.call(hook, seq[-1])
