"""Median C3 training-step time (B=256, T=128) of the library AUTOVC_HIP_LIB points at (for A/B
runs of two builds in alternating processes)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import onehot_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
B, T = 256, 128
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
ae.configure_optimizer()
X = torch.from_numpy(synthetic_mel(3, B, T)).to(dev)
c = torch.from_numpy(onehot_embedding(B)).to(dev)
for _ in range(2):
    ae.train_step(X, c)
ts = []
for _ in range(8):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ae.train_step(X, c)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print(f"{os.environ.get('AUTOVC_HIP_LIB', 'in-tree')}: median {np.median(ts):.2f} ms per C3 step")
