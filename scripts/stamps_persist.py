"""Phase breakdown of the weight-stationary lstm2 launch (lstm_persist.hip) from the diagnostic
stamps build (make stamps -> diag/libautovc_hip_stamps.so).

Per (workgroup, step): [0] step start -> [1] poll matched -> [2] acquire + barrier -> [3] MFMA loop
done (wave 0) -> [4] LDS reduce done -> [5] epilogue stored + drained (then the counter add).
Also: hand-off latency = poll match of a consumer at t - last producer's [5] at t-1."""
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

B, T, NCB = 64, 128, 64
lib = _lib.load()
if len(sys.argv) > 1:
    _lib.call("avc_lstm_persist_tune", int(sys.argv[1]))
if len(sys.argv) > 2:  # diagnostic bits (timing experiments; outputs not meaningful)
    lib.avc_debug_persist_diag.argtypes = [ctypes.c_int]
    lib.avc_debug_persist_diag(int(sys.argv[2]))
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
buf = torch.zeros(3 * NCB * T * 8, dtype=torch.int64, device=dev)
lib.avc_debug_stamps_persist(ctypes.c_void_p(buf.data_ptr()))
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.no_grad():
    ev0.record()
    ae(x, c, c)
    ev1.record()
torch.cuda.synchronize()
lib.avc_debug_stamps_persist(ctypes.c_void_p(0))
st = buf.view(3, NCB, T, 8).cpu().numpy().astype(np.int64)
rt = st[:, :, :, 6:8]  # s_memrealtime (100 MHz) at publish / poll match
span_rt = rt[..., 0].max() - rt[..., 1][rt[..., 1] > 0].min()
per_step = np.median(np.diff(st[0, :, 4:T - 4, 5], axis=1))
per_step_rt = np.median(np.diff(st[0, :, 4:T - 4, 6], axis=1))
clk = per_step / (per_step_rt * 10e-9) / 1e9
print(f"forward {ev0.elapsed_time(ev1):.3f} ms; persistent span {span_rt / 100:.1f} us (realtime); "
      f"s_memtime clock ~{clk:.2f} GHz")
names = ["poll wait", "acquire+barrier", "mfma loop", "lds reduce", "epilogue+drain"]
for L in range(3):
    s = st[L, :, 4:T - 4, :]
    ph = [np.median(s[:, :, i + 1] - s[:, :, i]) for i in range(5)]
    step = np.median(np.diff(st[L, :, 4:T - 4, 5], axis=1))
    print(f"slot {L}: per-step median ticks: " + ", ".join(f"{n} {v:.0f}" for n, v in zip(names, ph)) +
          f"; step-to-step {step:.0f}")
# hand-off: slot 0 at t polls cnt0[t-1]: last producer's publish at t-1 -> each consumer's match at t
pub = rt[0, :, :, 0].max(axis=0)        # [T] last slot-0 publish per step (realtime)
match = rt[0, :, 1:, 1]                 # [NCB][T-1]
lat = (match - pub[None, :-1]) * 10.0   # ns
print(f"slot0 hand-off (last publish t-1 -> poll match t): median {np.median(lat):.0f} ns, "
      f"p1 {np.percentile(lat, 1):.0f}, p99 {np.percentile(lat, 99):.0f} ns")
skew = (rt[0, :, 4:T - 4, 0].max(axis=0) - rt[0, :, 4:T - 4, 0].min(axis=0)) * 10.0
print(f"slot0 publish skew across workgroups per step: median {np.median(skew):.0f} ns")
for L in range(3):
    d = np.diff(rt[L, :, 4:T - 4, 0], axis=1) * 10.0
    print(f"slot {L}: step-to-step (realtime) median {np.median(d):.0f} ns")
