"""Bit-identity of two library builds on the conversion forwards: C2 (B=64, T=128), a ragged C5
batch (B=32, T=1024) and B=1 / B=3 cases, train-mode BN, plus the per-layer autograd path's
gradients at B=64.  Run once per build (AUTOVC_HIP_LIB=...) with an output path, then
`python scripts/compare_train.py --diff a.pt b.pt` compares the saved tensors."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
out = {}
for B, T in ((64, 128), (32, 1024), (1, 128), (3, 96)):
    x = synthetic_mel(40 + B, B, T)
    if T == 1024:
        for i, n in enumerate(np.random.default_rng(2).integers(256, T + 1, size=B)):
            x[i, :, n:] = 0.0
    x = torch.from_numpy(x).to(dev)
    co = torch.from_numpy(synthetic_embedding(41 + B, B)).to(dev)
    ct = torch.from_numpy(synthetic_embedding(42 + B, B)).to(dev)
    with torch.no_grad():
        for k, o in zip(("mel", "post", "codes"), ae(x, co, ct)):
            out[f"B{B}_T{T}_{k}"] = o.detach().cpu()
x = torch.from_numpy(synthetic_mel(7, 64, 128)).to(dev).requires_grad_(True)
co = torch.from_numpy(synthetic_embedding(8, 64)).to(dev)
mel, post, codes = ae(x, co, co)
(post.square().mean() + mel.abs().mean() + codes.square().mean()).backward()
out["dx"] = x.grad.detach().cpu()
for n, p in ae.named_parameters():
    if p.grad is not None:
        out["g_" + n] = p.grad.detach().cpu()
torch.save(out, sys.argv[1])
