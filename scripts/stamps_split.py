"""Phase breakdown of split-fp16 LSTM step launches from the diagnostic stamps build.

Phases per wave: [0] start -> [1] first chunk landed -> [2] MFMA loop done -> [3] LDS reduce done
-> [4] slab published + ticket (split-K only) -> [5] slabs reduced -> [6] epilogue done.
s_memtime ticks (100 MHz constant clock on gfx950? see the printed span vs event time)."""
import ctypes
import os
import sys

REPO = __file__.rsplit("/", 2)[0]
os.environ["AUTOVC_HIP_LIB"] = os.path.join(REPO, "diag", "libautovc_hip_stamps.so")
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

lib = _lib.load()
lib.avc_debug_stamps_split.argtypes = [ctypes.c_void_p, ctypes.c_long]
dev = torch.device("cuda:0")
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, 64, 128)).to(dev)
c = torch.from_numpy(synthetic_embedding(101, 64)).to(dev)
with torch.no_grad():
    ae(x, c, c)
torch.cuda.synchronize()
buf = torch.zeros(65536 * 8, dtype=torch.int64, device=dev)
names = ["first chunk", "mfma loop", "lds reduce", "slab+ticket", "slab reduce", "epilogue"]
for arg in sys.argv[1:] or ["0:0"]:
    ks, nc, r64 = (int(v) for v in (arg + ":0").split(":")[:3])
    _lib.call("avc_lstm_split_tune", ks, nc, r64)
    for name, idx in [("lstm1 H=512 step 64", 64), ("lstm2 pair step 64", 128 + 64)]:
        buf.zero_()
        lib.avc_debug_stamps_split(ctypes.c_void_p(buf.data_ptr()), idx)
        with torch.no_grad():
            ae(x, c, c)
        torch.cuda.synchronize()
        st = buf.view(65536, 8)[:, :7].cpu().numpy().astype(np.int64)
        st = st[st[:, 0] > 0]
        if len(st) == 0:
            print(name, "no stamps")
            continue
        t0 = st[:, 0].min()
        end = np.where(st[:, 6] > 0, st[:, 6], st[:, 4])
        print(f"kslice={ks} nc={nc} {name}: waves {len(st)}  span {end.max() - t0} ticks; "
              f"reducer waves {(st[:, 6] > 0).sum()}")
        for i, ph in enumerate(names):
            a, b = st[:, i], st[:, i + 1]
            ok = (a > 0) & (b > 0)
            if i == 4:  # slab reduce starts at the ticket
                a, b = st[:, 4], st[:, 5]
                ok = (a > 0) & (b > 0)
            elif i == 3:
                ok = (a > 0) & (b > 0)
            v = (b - a)[ok]
            if len(v):
                print(f"   {ph:14s} median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}  max {v.max():8.0f}  n {len(v)}")
        print(f"   wave start offset median {np.median(st[:, 0] - t0):8.0f}  max {(st[:, 0] - t0).max():8.0f}")
_lib.call("avc_lstm_split_tune", 0, 0, 0)
