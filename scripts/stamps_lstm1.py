"""Phase breakdown of the one-layer persistent recurrence (decoder.lstm1, lstm_persist.hip) from
the diagnostic stamps build (make stamps).  lstm2 is forced onto the step kernels so only lstm1
writes stamps.  Phases as scripts/stamps_persist.py."""
import ctypes
import os
import sys

REPO = __file__.rsplit("/", 2)[0]
os.environ["AUTOVC_HIP_LIB"] = os.environ.get("AVC_STAMPS_LIB", os.path.join(REPO, "diag", "libautovc_hip_stamps.so"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

# AVC_STAMPS_BT="32,1024" for C5's shape (default C2: 64, 128)
B, T = (int(v) for v in os.environ.get("AVC_STAMPS_BT", "64,128").split(","))
NWG = 256  # (the XCD-local grid is linear: 8 x ncb workgroups, bid = residue + 8 x column block)
lib = _lib.load()
_lib.call("avc_lstm_persist_layers", 1)
lib.avc_debug_stamps_persist.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
c = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
with torch.no_grad():
    ae(x, c, c)
torch.cuda.synchronize()
buf = torch.zeros(NWG * T * 8, dtype=torch.int64, device=dev)
names = ["poll wait", "acquire+barrier", "mfma loop", "lds reduce", "epilogue+drain"]


def measure(label):
    buf.zero_()
    lib.avc_debug_stamps_persist(ctypes.c_void_p(buf.data_ptr()))
    with torch.no_grad():
        ae(x, c, c)
    torch.cuda.synchronize()
    lib.avc_debug_stamps_persist(ctypes.c_void_p(0))
    st = buf.view(NWG, T, 8).cpu().numpy().astype(np.int64)
    st = st[(st[:, 4:T - 4, :6] != 0).all(axis=(1, 2))]  # the recurrent workgroups (every stamp written)
    s = st[:, 4:T - 4, :]
    ph = [np.median(s[:, :, i + 1] - s[:, :, i]) for i in range(5)]
    step = np.median(np.diff(st[:, 4:T - 4, 5], axis=1))
    d = np.diff(st[:, 4:T - 4, 6], axis=1) * 10.0
    print(f"{label}: lstm1 per-step median ticks: " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, ph)) +
          f"; step-to-step {step:.0f} ticks, realtime {np.median(d):.0f} ns", flush=True)


measure("default")
# further measurements after each tuning call: "depth=1" -> avc_lstm_persist_depth(1); a bare
# integer is an avc_lstm_persist_qwait mask
for arg in sys.argv[1:]:
    name, val = arg.split("=") if "=" in arg else ("qwait", arg)
    _lib.call(f"avc_lstm_persist_{name}", int(val))
    measure(arg)
