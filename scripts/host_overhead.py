"""Host-side submission time of the fused forward vs its GPU time (is the host the bottleneck?)."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
m = AutoEncoder(device=dev, verbose=False)
m.load_state_dict(torch_state_dict(0))
m.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, 64, 128)).to(dev)
c = torch.from_numpy(synthetic_embedding(101, 64)).to(dev)
with torch.no_grad():
    for _ in range(3):
        m(x, c, c)
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        m(x, c, c)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host submit {1000 * (t1 - t0) / n:.3f} ms/fwd, wall {1000 * (t2 - t0) / n:.3f} ms/fwd")
    t0 = time.perf_counter()
    for _ in range(200):
        m._gen_params()
    print(f"_gen_params {1e6 * (time.perf_counter() - t0) / 200:.1f} us")
