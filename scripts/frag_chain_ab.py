"""A/B of the conv -> conv split-image hand-over (ops._FRAG_CHAIN) on the C3 training step
(B=256, T=128), alternating in one process: median ms per step of each setting per round."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import ops  # noqa: E402
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
for _ in range(3):
    ae.train_step(X, c)
res = {False: [], True: []}
for rnd in range(4):
    for chain in (False, True):
        ops._FRAG_CHAIN = chain
        ae.train_step(X, c)
        ts = []
        for _ in range(6):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ae.train_step(X, c)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        res[chain].append(float(np.median(ts)))
        print(f"round {rnd} chain={chain}: {res[chain][-1]:.3f} ms", flush=True)
ops._FRAG_CHAIN = True
print(f"median: off {np.median(res[False]):.3f} ms, on {np.median(res[True]):.3f} ms")
