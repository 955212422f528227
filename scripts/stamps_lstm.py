"""Phase breakdown of LSTM step launches from the diagnostic stamps build (diag/*.so).

Phases per wave: [0] start -> [1] first operand group landed -> [2] MFMA loop done ->
[3] cross-wave reduction done -> [4] epilogue done.  s_memtime ticks at the shader clock."""
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
lib.avc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_long]
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
# launch indices inside one forward: 0..127 lstm1 (H=512), 128.. lstm2 pair (128 = t0 only, 129.. pairs)
for name, idx in [("lstm1 H=512 step 64", 64), ("lstm2 pair step 64", 128 + 64), ("lstm2 first (layer0 only)", 128 + 1 - 1)]:
    buf.zero_()
    lib.avc_debug_stamps(ctypes.c_void_p(buf.data_ptr()), idx)
    with torch.no_grad():
        ae(x, c, c)
    torch.cuda.synchronize()
    st = buf.view(65536, 8)[:, :5].cpu().numpy().astype(np.int64)
    st = st[st[:, 0] > 0]
    if len(st) == 0:
        print(name, "no stamps")
        continue
    t0 = st[:, 0].min()
    rel = st - t0
    d = np.diff(st, axis=1)
    print(f"{name}: waves {len(st)}  span {rel[:, 4].max()} ticks")
    for i, ph in enumerate(["loads(first group)", "mfma loop", "reduce", "epilogue"]):
        v = d[:, i]
        print(f"   {ph:20s} median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}  max {v.max():8.0f}")
    print(f"   wave start offset   median {np.median(rel[:, 0]):8.0f}  max {rel[:, 0].max():8.0f}")
