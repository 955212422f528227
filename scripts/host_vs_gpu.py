"""Host vs device time of the C2 fused forward (bench.py's step): per-call host time without a
sync, wall time of N back-to-back calls, and the device time between events recorded before the
first and after the last call.  Tells whether the host keeps the GPU fed."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
B, T, N = 64, 128, 30
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
with torch.no_grad():
    for _ in range(5):
        ae(x, co, ct)
    torch.cuda.synchronize()
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        host = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(N):
            h0 = time.perf_counter()
            ae(x, co, ct)
            host.append(time.perf_counter() - h0)
        e1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        host.sort()
        print(f"rep {rep}: wall {1e3 * wall / N:.3f} ms/step, device {e0.elapsed_time(e1) / N:.3f} ms/step, "
              f"host call median {1e3 * host[N // 2]:.3f} ms, max {1e3 * host[-1]:.3f} ms, first {1e3 * host[0]:.3f}")
