"""Run-to-run determinism of forward and backward (same process, same inputs, same init)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import onehot_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
sd = torch_state_dict(0)
X = torch.from_numpy(synthetic_mel(30, 4, 128)).to(dev)
c = torch.from_numpy(onehot_embedding(4)).to(dev)
runs = []
for r in range(3):
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(sd)
    ae.to(dev).train()
    md, mp, mc = ae(X, c, c)
    loss = ae._loss(X, c, md, mp, mc)
    loss.backward()
    torch.cuda.synchronize()
    runs.append(({"mel": md.detach().clone(), "post": mp.detach().clone(), "codes": mc.detach().clone(),
                  "loss": loss.detach().clone()},
                 {k: p.grad.detach().clone() for k, p in ae.named_parameters()}))
for r in (1, 2):
    for k in runs[0][0]:
        d = (runs[r][0][k] - runs[0][0][k]).abs().max().item()
        if d:
            print(f"run {r} fwd {k} differs: {d:.3e}")
    bad = [(k, (runs[r][1][k] - runs[0][1][k]).abs().max().item()) for k in runs[0][1]]
    bad = [b for b in bad if b[1] > 0]
    print(f"run {r}: {len(bad)} parameter grads differ", bad[:12])
