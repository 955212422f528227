"""One-layer persistent LSTM (lstm_persist.hip, one-layer form) against the launch-per-step
kernel over batch sizes and H; reports give-ups per shape (debug aid)."""
import ctypes
import sys
import torch
sys.path.insert(0, ".")
from autovc_amd import _lib, ops

dev = torch.device("cuda:0")
torch.manual_seed(0)


def giveups():
    n = ctypes.c_long(0)
    _lib.call("avc_lstm_persist_status", ctypes.byref(n))
    return n.value


T = 128
for H, din in ((512, 320), (1024, 512)):
    wi = (torch.rand(4 * H, din, device=dev) - 0.5) * 0.1
    wh = (torch.rand(4 * H, H, device=dev) - 0.5) * 0.1
    bi = torch.rand(4 * H, device=dev) * 0.1
    bh = torch.rand(4 * H, device=dev) * 0.1
    for B in (16, 32, 48, 64, 96, 128, 192, 256):
        x = torch.rand(T * B, din, device=dev)
        res = {}
        for mode in (0, 2):
            _lib.call("avc_lstm_persist_tune", mode)
            for save in (False, True):
                g0 = giveups()
                try:
                    y = ops.LSTMLayer.apply(x, wi, wh, bi, bh, T, B, save)
                    torch.cuda.synchronize()
                    err = ""
                except RuntimeError as e:
                    y, err = None, str(e)[:60]
                res[(mode, save)] = (y, giveups() - g0, err)
        _lib.call("avc_lstm_persist_tune", 2)
        ref = res[(0, False)][0]
        line = []
        for k, (y, gv, err) in res.items():
            d = float((y - ref).abs().max()) if y is not None else float("nan")
            line.append(f"mode{k[0]} save{int(k[1])}: giveups {gv} maxd {d:.1e} {err}")
        print(f"H={H} B={B}: " + " | ".join(line), flush=True)
