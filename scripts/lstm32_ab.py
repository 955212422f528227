"""A/B of the encoder BiLSTM recurrence (avc_lstm32_tune) inside the fused C2 forward: per-launch
time of the lstm32 timing class per mode, and the largest output difference against mode 0."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
B, T = (int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (64, 128)))
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(5, B, T)).to(dev)
co = torch.from_numpy(synthetic_embedding(6, B)).to(dev)
outs = {}
for mode in (0, 1, 0, 1):
    _lib.call("avc_lstm32_tune", mode)
    _lib.timing_enable(["lstm32"])
    _lib.timing_reset()
    with torch.no_grad():
        for _ in range(5):
            o = [t.clone() for t in ae(x, co, co)]
    torch.cuda.synchronize()
    r = _lib.timing_read("lstm32")
    _lib.timing_enable([])
    outs[mode] = o
    print(f"mode {mode}: lstm32 {1e3 * r['ms'] / max(r['launches'], 1):.1f} us per launch ({r['launches']} launches)",
          flush=True)
d = max((a - b).abs().max().item() for a, b in zip(outs[0], outs[1]))
print(f"max|mode1 - mode0| over mel / mel_post / codes: {d:.2e}")
_lib.call("avc_lstm32_tune", 1)
