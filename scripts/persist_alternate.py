"""Stale-read check for the persistent recurrences' hand-off forms: references for two different
input batches from the acquire form (avc_lstm_persist_tune(1)), then N forwards alternating the two
batches under the form given in argv[1] (default 2 = sc1 loads), each compared with its reference.
Same-input repeats cannot see a stale read (the stale bytes are equal); alternating inputs can."""
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
B, T, N = 64, 128, 24
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
xs = [torch.from_numpy(synthetic_mel(s, B, T)).to(dev) for s in (1, 2)]
co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
refs = []
with torch.no_grad():
    _lib.call("avc_lstm_persist_tune", 1)
    _lib.timing_enable(["lstm2_persist"])  # eager launches for the references
    for x in xs:
        refs.append([o.clone() for o in ae(x, co, ct)])
    _lib.timing_enable([])
    _lib.call("avc_lstm_persist_tune", mode)
    bad = 0
    for i in range(N):
        k = i % 2
        out = ae(xs[k], co, ct)
        torch.cuda.synchronize()
        d = max((a - b).abs().max().item() for a, b in zip(out, refs[k]))
        bad += d != 0
        print(f"mode {mode} call {i} input {k}: max|d| {d:.2e}", flush=True)
print(f"mode {mode}: {bad} of {N} alternating calls differ from the acquire-form references")
_lib.call("avc_lstm_persist_tune", 2)
