"""A/B of training-step options at C3 (B=256, T=128): in-place parameter gradients
(AutoEncoder.inplace_grads) on / off, alternating, median step time of each."""
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
res = {True: [], False: []}
for rep in range(6):
    for mode in (True, False):
        ae.inplace_grads = mode
        ae.train_step(X, c)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            ae.train_step(X, c)
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) / 3 * 1e3)
for mode in (True, False):
    print(f"inplace_grads={mode}: median {np.median(res[mode]):.2f} ms  ({', '.join(f'{v:.2f}' for v in res[mode])})")
