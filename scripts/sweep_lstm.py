"""Sweep the LSTM step-kernel configuration (rows per block x waves) on the GPU."""
import itertools
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from autovc_amd import _lib, ops  # noqa: E402


def run(din, H, B, T, bwd):
    dev = torch.device("cuda:0")
    k = 1.0 / H ** 0.5
    x = torch.rand(T * B, din, device=dev)
    wi = ((torch.rand(4 * H, din, device=dev) * 2 - 1) * k).requires_grad_(bwd)
    wh = ((torch.rand(4 * H, H, device=dev) * 2 - 1) * k).requires_grad_(bwd)
    bi = torch.zeros(4 * H, device=dev, requires_grad=bwd)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    _lib.timing_enable(["lstm_step_fwd", "lstm_step_bwd"])
    for mb, nw in itertools.product([16, 32, 64], [2, 4, 8]):
        _lib.call("avc_lstm_tune", mb, nw)
        for rep in range(3):
            _lib.timing_reset()
            if bwd:
                y = ops.LSTMLayer.apply(x, wi, wh, bi, bi, T, B, True)
                y.backward(torch.ones_like(y))
            else:
                with torch.no_grad():
                    ops.LSTMLayer.apply(x, wi, wh, bi, bi, T, B, False)
            torch.cuda.synchronize()
        r = _lib.timing_read("lstm_step_bwd" if bwd else "lstm_step_fwd")
        res[f"mb{mb}_nw{nw}"] = round(1000 * r["ms"] / max(1, r["launches"]), 2)
    _lib.call("avc_lstm_tune", 0, 0)
    _lib.timing_enable([])
    return res


if __name__ == "__main__":
    out = {}
    for (din, H, B, bwd) in [(1024, 1024, 64, False), (320, 512, 64, False), (1024, 1024, 256, False),
                             (1024, 1024, 64, True), (1024, 1024, 256, True)]:
        key = f"{'bwd' if bwd else 'fwd'} H={H} B={B}"
        out[key] = run(din, H, B, 128, bwd)
        print(key, json.dumps(out[key]), flush=True)
