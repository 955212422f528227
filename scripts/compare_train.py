"""Bit-identity of two library builds on C3 training steps (B=256, T=128): run once per build
(AUTOVC_HIP_LIB=...) with an output path, then compare the saved tensors with --diff.
    AUTOVC_HIP_LIB=a.so python scripts/compare_train.py out_a.pt; python scripts/compare_train.py out_b.pt
    python scripts/compare_train.py --diff out_a.pt out_b.pt"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
if sys.argv[1] == "--diff":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    bad = 0
    for k in a:
        same = torch.equal(a[k], b[k])
        bad += not same
        print(f"{k}: max|d| {(a[k] - b[k]).abs().max().item():.3e} {'bit-identical' if same else 'DIFFERENT'}")
    sys.exit(1 if bad else 0)
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
out = {}
for i in range(2):
    loss, norm = ae.train_step(X, c)
    out[f"loss{i}"] = loss.detach().cpu().reshape(1)
    out[f"norm{i}"] = norm.detach().cpu().reshape(1)
out["params"] = torch.cat([p.detach().reshape(-1) for p in ae.parameters()]).cpu()
torch.save(out, sys.argv[1])
