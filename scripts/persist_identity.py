"""Where do the persistent recurrences (lstm_persist.hip) and the step launches (lstm_split.hip)
differ?  (1) one LSTM layer through the C ABI (avc_lstm_forward) at several shapes, y / gates / c
compared exactly between avc_lstm_persist_tune(0) and (2); (2) the fused C2 forward on two input
sets.  Prints max |d| per output."""
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402

from autovc_amd import _lib, ops  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(5)


def layer(mode, T, B, din, H, x, w):
    _lib.call("avc_lstm_persist_tune", mode)
    y = torch.empty(T * B, H, device=dev)
    gates, c = ops._lstm_fwd(x, *w, y, 0, H, False, True, T, B)
    torch.cuda.synchronize()
    return y, gates, c


for (T, B, din, H) in [(128, 64, 320, 512), (16, 64, 320, 512), (8, 16, 64, 512), (8, 64, 512, 1024)]:
    x = (torch.rand(T * B, din, generator=g) - 0.5).to(dev)
    s = 1.0 / H ** 0.5
    w = [((torch.rand(*shape, generator=g) * 2 - 1) * s).to(dev)
         for shape in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
    r0 = layer(0, T, B, din, H, x, w)
    r2 = layer(2, T, B, din, H, x, w)
    d = [(a - b).abs().max().item() for a, b in zip(r0, r2)]
    # first step / first row where y differs
    bad = (r0[0] != r2[0]).view(T, B, H).any(dim=2).nonzero()
    print(f"layer T={T} B={B} din={din} H={H}: max|d| y {d[0]:.3e} gates {d[1]:.3e} c {d[2]:.3e}; "
          f"first differing (t, b): {bad[0].tolist() if len(bad) else None}", flush=True)

for seed in (1, 104):
    B, T = 64, 128
    ae = AutoEncoder(device=dev, verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    ae.to(dev).train()
    x = torch.from_numpy(synthetic_mel(seed, B, T)).to(dev)
    co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
    ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
    outs = {}
    for mode in (0, 2):
        _lib.call("avc_lstm_persist_tune", mode)
        with torch.no_grad():
            outs[mode] = [o.clone() for o in ae(x, co, ct)]
    d = [(a - b).abs().max().item() for a, b in zip(outs[0], outs[2])]
    print(f"fused forward seed {seed}: max|d| mel {d[0]:.3e} mel_post {d[1]:.3e} codes {d[2]:.3e}", flush=True)
_lib.call("avc_lstm_persist_tune", 2)
