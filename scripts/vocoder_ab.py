"""A/B of the WaveRNN sample loop: per-step graph chunks (avc_wavernn_persist 0) against the
persistent loop (1), alternating in one process on the bench's 10 s utterance (bench.py --mode
vocoder: 801 mel frames, batched target 11000 / overlap 550 -> 20 fold rows x 12100 steps).
Prints the median generate() time per mode and whether the waveforms are bit-identical."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib  # noqa: E402
from autovc_amd.wavernn import WaveRNN  # noqa: E402
from autovc_amd.weights import synthetic_mel, wavernn_state_dict  # noqa: E402

dev = torch.device("cuda:0")
T = 10 * 22050 // 275
net = WaveRNN(device=dev)
net.load_state_dict(wavernn_state_dict(0))
mel = torch.from_numpy(synthetic_mel(31, 1, T)).to(dev)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
times, waves = {0: [], 1: []}, {}
for r in range(reps + 1):
    for mode in (0, 1):
        _lib.call("avc_wavernn_persist", mode)
        torch.manual_seed(7)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w = net.generate(mel)
        dt = time.perf_counter() - t0
        if r > 0:
            times[mode].append(dt)
        waves[mode] = w
        print(f"rep {r} persist={mode}: {1e3 * dt:.1f} ms", flush=True)
_lib.call("avc_wavernn_persist", 1)  # (the default)
audio_s = (T - 1) * 275 / 22050
for mode in (0, 1):
    med = float(np.median(times[mode]))
    print(f"persist={mode}: median {1e3 * med:.1f} ms per generate = {audio_s / med:.2f} audio-s/s, "
          f"{1e6 * med / 12100:.1f} us per sample step")
print("waveforms bit-identical:", bool(np.array_equal(waves[0], waves[1])),
      "max |d|", float(np.abs(waves[0] - waves[1]).max()))
