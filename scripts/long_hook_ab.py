"""A/B of one library hook (argv[1]; values argv[2:]) on bench.py's C5 long-form forward (B = 32,
ragged lengths <= 1024, zero-padded; the exact bench batch), alternating in one process: median
ms per forward over 10 steps after 3 warm-up steps, per value."""
import sys
import time
import types

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import bench  # noqa: E402
from autovc_amd import _lib  # noqa: E402

hook = sys.argv[1]
vals = [int(v) for v in sys.argv[2:]] or [0, 1]
dev = torch.device("cuda:0")
args = types.SimpleNamespace(batch=None, frames=128, cpu_seconds=0)
m = bench.setup_long(args, dev, 0)
res = {v: [] for v in vals}
for rep in range(4):
    for v in vals:
        _lib.call(hook, v)
        for _ in range(3):
            m["step"]()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            m["step"]()
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) / 10 * 1e3)
for v in vals:
    print(f"C5 {hook}={v}: median {np.median(res[v]):.3f} ms per forward ({', '.join(f'{t:.3f}' for t in res[v])})", flush=True)
