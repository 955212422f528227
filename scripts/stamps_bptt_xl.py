"""Phase breakdown of the XCD-local BPTT (bptt_xl_kernel, H = 512) from the diagnostic stamps
build (make stamps): one LSTMLayer backward at C3's lstm1 shape (B = 256, T = 128, din = 320).
Slots per (workgroup, step): 0 step start, 1 phase-A MFMAs done, 2 partials drained + barrier,
3 every partial of the group published (poll + barrier), 4 partials summed, 5 dG formed and
stored, 6 row-max barrier, 7 split dG in LDS (step end)."""
import ctypes
import os
import sys

REPO = __file__.rsplit("/", 2)[0]
os.environ["AUTOVC_HIP_LIB"] = os.environ.get("AVC_STAMPS_LIB", os.path.join(REPO, "diag", "libautovc_hip_stamps.so"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from autovc_amd import _lib, ops  # noqa: E402

B, T, din, H = 256, 128, 320, 512
lib = _lib.load()
lib.avc_debug_stamps_persist.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(1)
k = 1.0 / H ** 0.5
ws = [((torch.rand(*s, generator=g) * 2 - 1) * k).to(dev).requires_grad_(True)
      for s in [(4 * H, din), (4 * H, H), (4 * H,), (4 * H,)]]
x = (torch.randn(T * B, din, generator=g) * 0.5).to(dev).requires_grad_(True)
dy = torch.randn(T * B, H, generator=g).to(dev)
buf = torch.zeros(256 * T * 8, dtype=torch.int64, device=dev)
names = ["A mfma", "A store+drain", "publish->all in", "partial loads", "gate math+store", "rowmax barrier", "split+barrier"]
for rep in range(3):
    y = ops.LSTMLayer.apply(x, *ws, T, B, True)
    torch.cuda.synchronize()
    buf.zero_()
    lib.avc_debug_stamps_persist(ctypes.c_void_p(buf.data_ptr()))
    y.backward(dy)
    torch.cuda.synchronize()
    lib.avc_debug_stamps_persist(ctypes.c_void_p(0))
    st = buf.view(256, T, 8).cpu().numpy().astype(np.int64)
    s = st[:, 4:T - 4, :]
    ph = [np.median(s[:, :, i + 1] - s[:, :, i]) for i in range(7)]
    step = np.median(np.diff(st[:, 4:T - 4, 0], axis=1))
    print(f"rep {rep}: per-step median ticks: " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, ph)) +
          f"; step-to-step {step:.0f}", flush=True)
