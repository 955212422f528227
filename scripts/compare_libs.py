"""Bit-identity of two library builds on the C2 forward (and a conv+BN layer): run this script
once per build (AUTOVC_HIP_LIB=...) with an output path, then compare the saved tensors.
    AUTOVC_HIP_LIB=a.so python scripts/compare_libs.py out_a.pt; ... out_b.pt; python scripts/compare_libs.py --diff out_a.pt out_b.pt"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
if sys.argv[1] == "--diff":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    for k in a:
        d = (a[k] - b[k]).abs().max().item()
        print(f"{k}: max|d| {d:.3e} {'bit-identical' if torch.equal(a[k], b[k]) else 'DIFFERENT'}")
    sys.exit(0)
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, 64, 128)).to(dev)
c = torch.from_numpy(synthetic_embedding(101, 64)).to(dev)
with torch.no_grad():
    mel, post, codes = ae(x, c, c)
torch.save({"mel": mel.cpu(), "mel_post": post.cpu(), "codes": codes.cpu()}, sys.argv[1])
