"""A/B of the one-layer persistent form's h hand-off (avc_lstm_persist_granules): the fused
forward at C2 (B=64, T=128), a C5-like shape (B=32, T=1024) and the C3 training shape (B=256,
T=128, with autograd: gates and cell state saved), alternating 0 / 1 in one process; ms per
forward, lstm1 us per launch from the library's timing events, and a bit-identity check of the
outputs against the first run."""
import ctypes
import sys
import time

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
seq = [int(v) for v in sys.argv[1:]] or [0, 1, 0, 1]
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
for B, T, grad in ((64, 128, False), (32, 1024, False), (256, 128, True)):
    x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
    co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
    ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
    ref = None
    for q in seq:
        _lib.call("avc_lstm_persist_granules", q)
        with torch.set_grad_enabled(grad):
            for _ in range(3):
                out = ae(x, co, ct)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                out = ae(x, co, ct)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 10 * 1e3
            _lib.timing_enable(["lstm1_persist"])
            _lib.timing_reset()
            for _ in range(5):
                ae(x, co, ct)
            torch.cuda.synchronize()
            k1 = _lib.timing_read("lstm1_persist")
            _lib.timing_enable([])
        out = [o.detach() for o in out]
        if ref is None:
            ref = [o.clone() for o in out]
        same = all(torch.equal(a, b) for a, b in zip(out, ref))
        print(f"B={B} T={T} grad={grad} granules {q}: {ms:.3f} ms per forward; "
              f"lstm1 {1e3 * k1['ms'] / max(1, k1['launches']):.1f} us per launch; bit-identical {same}", flush=True)
g = ctypes.c_long(0)
_lib.call("avc_lstm_persist_status", ctypes.byref(g))
print("giveups", g.value)
_lib.call("avc_lstm_persist_granules", 1)
