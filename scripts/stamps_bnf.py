"""Phase breakdown of the fused Conv1d + BatchNorm epilogue (gemm.hip bnf_epilogue) from the
diagnostic build with -DAVC_GEMM_EPI_STAMPS (AUTOVC_HIP_LIB): the last 512 -> 512 conv of the C2
forward (postnet; B = 64, T = 128, train-mode BN; 256 workgroups of 128 x 128).  s_memtime per workgroup (thread 0):
0 K loop start, 1 K loop end, 2 act loop, 3 column partials stored, 4 drained + barrier,
5 column-tile wait done, 6 partials combined, 7 scale / shift, 8 tile staged, 9 outputs stored."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(3, 64, 128)).to(dev)
c = torch.from_numpy(synthetic_embedding(4, 64)).to(dev)
lib = _lib.load()
lib.avc_debug_epi_stamps.argtypes = [ctypes.c_void_p]
with torch.no_grad():
    for _ in range(5):
        ae(x, c, c)
torch.cuda.synchronize()
st = np.zeros((1024, 10), dtype=np.uint64)
lib.avc_debug_epi_stamps(ctypes.c_void_p(st.ctypes.data))
s = st[:256].astype(np.int64)
names = ["K loop", "act loop", "col partials", "drain+barrier", "tile wait", "combine", "scale/shift",
         "tile stage", "outputs"]
t0 = s[:, 0].min()
print(f"workgroups 256; K-loop end spread (max - min) {s[:, 1].max() - s[:, 1].min()} ticks; "
      f"first start -> last end {s[:, 9].max() - t0} ticks")
for i, n in enumerate(names):
    d = s[:, i + 1] - s[:, i]
    print(f"{n:14s} median {int(np.median(d)):7d}  p10 {int(np.percentile(d, 10)):7d}  p90 {int(np.percentile(d, 90)):7d} ticks")
