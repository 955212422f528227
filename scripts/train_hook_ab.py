"""A/B of one library tuning hook (argv[1], e.g. avc_bn_fuse; values argv[2:]) on the C3 training
step (B = 256, T = 128), alternating the values in one process: median ms per step of each, and
the loss of one step from the same parameters under each value (the hooks compared here are
bit-identical options, so the losses must agree)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import onehot_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
hook = sys.argv[1]
vals = [int(v) for v in sys.argv[2:]] or [0, 1]
B, T = 256, 128
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
ae.configure_optimizer()
X = torch.from_numpy(synthetic_mel(3, B, T)).to(dev)
c = torch.from_numpy(onehot_embedding(B)).to(dev)
res = {v: [] for v in vals}
for rep in range(5):
    for v in vals:
        _lib.call(hook, v)
        ae.train_step(X, c)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            ae.train_step(X, c)
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) / 3 * 1e3)
ae.check_health()
for v in vals:
    print(f"C3 {hook}={v}: median {np.median(res[v]):.2f} ms per step ({', '.join(f'{t:.2f}' for t in res[v])})", flush=True)
# one step's loss from identical parameters under each value
sd = {k: t.detach().clone() for k, t in ae.state_dict().items()}
for v in vals:
    _lib.call(hook, v)
    ae2 = AutoEncoder(device=dev, verbose=False)
    ae2.load_state_dict(sd)
    ae2.to(dev).train()
    ae2.configure_optimizer()
    loss, gnorm = ae2.train_step(X, c)
    print(f"{hook}={v}: loss {float(loss):.9g} grad norm {float(gnorm):.9g}", flush=True)
_lib.call(hook, vals[0])
