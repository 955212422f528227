"""Find the first per-layer op whose output holds NaN in the C2 layerwise forward (debug aid)."""
import sys
import torch
sys.path.insert(0, ".")
from autovc_amd import ops
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict

dev = torch.device("cuda:0")
B, T = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 128
names = ["FramesFromMel", "MelFromFrames", "ConvBNAct", "LSTMLayer", "BiLSTMLayer", "Codes", "DecoderInput", "Linear"]
seen = []
for n in names:
    cls = getattr(ops, n)
    orig = cls.apply

    def wrap(*a, _orig=orig, _n=n):
        out = _orig(*a)
        torch.cuda.synchronize()
        bad = torch.isnan(out).sum().item()
        ins = [x for x in a if torch.is_tensor(x) and x.is_floating_point()]
        inbad = [torch.isnan(x).sum().item() for x in ins]
        seen.append((_n, tuple(out.shape), bad, inbad))
        print(_n, tuple(out.shape), "nan:", bad, "inputs nan:", inbad, flush=True)
        return out
    cls.apply = staticmethod(wrap)

ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
ae.fused_autograd = False
x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
for grad in (True, False):
    print("---- grad", grad)
    with torch.set_grad_enabled(grad):
        ae(x, co, ct)
