"""N C2 forwards (B = 64, T = 128, whole-Generator fused path, graph replay) under the library hook
settings in argv[1] ("hook=value,hook=value" or "-"), for PMC passes of one configuration:
rocprofv3 --pmc FETCH_SIZE -- python3 scripts/fwd_hooks.py avc_lstm_persist_qwait=0 5"""
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
if len(sys.argv) > 1 and sys.argv[1] != "-":
    for kv in sys.argv[1].split(","):
        h, v = kv.split("=")
        _lib.call(h, int(v))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B, T = 64, 128
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
with torch.no_grad():
    for _ in range(n):
        ae(x, co, ct)
torch.cuda.synchronize()
ae.check_health()
print("done", sys.argv[1:])
