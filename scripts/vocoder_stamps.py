"""Where a step of the persistent WaveRNN loop goes (diagnostics, avc_debug_wavernn_stamps).

Runs generate() of the bench's 10 s utterance with the loop on and s_memrealtime stamps (100 MHz)
of the first N steps: per workgroup and op (IN1 / IN2 = the GRUs' input phases, FC1, FC2, OUT,
HID = next step's hidden-gate phase of both layers) the op's start, the end of its wait and its end.
Prints, averaged over steps 16..N-1, the step period and for each chain op: the wait's end
relative to the producer's last end (hand-off latency) and the op's duration after the wait."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib  # noqa: E402
from autovc_amd.wavernn import WaveRNN  # noqa: E402
from autovc_amd.weights import synthetic_mel, wavernn_state_dict  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
dev = torch.device("cuda:0")
T = 10 * 22050 // 275
net = WaveRNN(device=dev)
net.load_state_dict(wavernn_state_dict(0))
mel = torch.from_numpy(synthetic_mel(31, 1, T)).to(dev)
G = 256
_lib.call("avc_wavernn_persist", 1)
net.generate(mel)  # warm (regions, code)
buf = torch.zeros(G, N, 24, dtype=torch.int64, device=dev)
_lib.call("avc_debug_wavernn_stamps", buf.data_ptr(), N)
net.generate(mel)
torch.cuda.synchronize()
_lib.call("avc_wavernn_persist", 1)  # (the default)
st = buf.cpu().numpy().astype(np.float64) * 10.0 / 1000.0  # -> microseconds
HID, _, IN1, IN2, FC1, FC2, OUT = range(7)
names = ["HID", "-", "IN1", "IN2", "FC1", "FC2", "OUT"]
nfc, R = 64, 20
roles = {FC1: range(0, nfc), FC2: range(nfc, 2 * nfc), OUT: range(2 * nfc, 2 * nfc + R)}
wgs = {op: list(roles.get(op, range(G))) for op in range(7)}
steps = range(16, N - 1)


def col(op, k, i):  # k: 0 start, 1 wait end, 2 end; over the op's workgroups at loop step i
    v = st[wgs[op], i, 3 * op + k]
    return v[v > 0]


t0 = st[st > 0].min()
period = np.mean([col(IN1, 2, i + 1).max() - col(IN1, 2, i).max() for i in steps])
print(f"loop step period {period:.2f} us (steps 16..{N - 1})")
chain = [(IN1, OUT, -1), (IN2, IN1, 0), (FC1, IN2, 0), (FC2, FC1, 0), (OUT, FC2, 0)]
for op, prod, di in chain:
    hand = np.mean([np.median(col(op, 1, i)) - col(prod, 2, i + di).max() for i in steps])
    wait_spread = np.mean([col(op, 1, i).max() - col(op, 1, i).min() for i in steps])
    dur = np.mean([np.median(col(op, 2, i) - col(op, 1, i)) for i in steps])
    dur_max = np.mean([(col(op, 2, i) - col(op, 1, i)).max() for i in steps])
    pre = np.mean([np.median(col(op, 1, i) - col(op, 0, i)) for i in steps])
    print(f"{names[op]:4s}: hand-off from {names[prod]} last end -> median wait end {hand:6.2f} us "
          f"(spread over consumers {wait_spread:5.2f}); after the wait median {dur:5.2f} / max {dur_max:5.2f} us; "
          f"start -> wait end {pre:6.2f} us")
for op in (HID,):
    dur = np.mean([np.median(col(op, 2, i) - col(op, 0, i)) for i in steps])
    print(f"{names[op]}: start -> end median {dur:.2f} us")
np.save("gpurun_out/vocoder_stamps.npy", st)
