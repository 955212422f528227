"""Repeatability of the fused C2 forward with the persistent recurrences: N forwards back to back
(graph replays, or eager launches when argv[1] == "eager": per-launch timing forces the eager
path; "bump": graph replays with a config-epoch bump every 8 calls, i.e. drop + eager + recapture), each compared with the first eager result.  Prints the mismatching calls and their times."""
import ctypes
import sys
import time

sys.path.insert(0, __file__.rsplit("/", 2)[0])
import torch  # noqa: E402

from autovc_amd import _lib  # noqa: E402
from autovc_amd.auto_encoder import AutoEncoder  # noqa: E402
from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict  # noqa: E402

dev = torch.device("cuda:0")
B, T, N = 64, 128, 40
how = sys.argv[1] if len(sys.argv) > 1 else "graph"
if len(sys.argv) > 2 and how != "modes":
    _lib.call("avc_lstm_persist_depth", int(sys.argv[2]))
if len(sys.argv) > 3 and how != "modes":
    _lib.call("avc_lstm_persist_tune", int(sys.argv[3]))
if len(sys.argv) > 4 and how != "modes":
    _lib.call("avc_lstm_persist_layers", int(sys.argv[4]))
ae = AutoEncoder(device=dev, verbose=False)
ae.load_state_dict(torch_state_dict(0))
ae.to(dev).train()
x = torch.from_numpy(synthetic_mel(1, B, T)).to(dev)
co = torch.from_numpy(synthetic_embedding(101, B)).to(dev)
ct = torch.from_numpy(synthetic_embedding(201, B)).to(dev)
with torch.no_grad():
    ref = [o.clone() for o in ae(x, co, ct)]
    if how == "eager":
        _lib.timing_enable(["lstm1_persist"])
    bad = []
    if how == "nosync":  # persist_modes.py's pattern: blocks of bump + 23 calls with no host sync
        for blk in range(4):
            _lib.call("avc_lstm_persist_depth", int(sys.argv[2]) if len(sys.argv) > 2 else 2)
            for _ in range(23):
                out = ae(x, co, ct)
            torch.cuda.synchronize()
            d = max((a - b).abs().max().item() for a, b in zip(out, ref))
            print(f"nosync block {blk}: max|d| {d:.2e}", flush=True)
        N = 0
    if how == "modes":  # persist_modes.py exactly, plus status and an eager recompute per block
        specs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "2:2", "2:2", "2:2"]
        eager_check = not (len(sys.argv) > 3 and sys.argv[3] == "noeager")
        force_eager = len(sys.argv) > 4 and sys.argv[4] == "eager"   # timing on => no graph
        sync_each = len(sys.argv) > 4 and sys.argv[4] == "synceach"
        if force_eager:
            _lib.timing_enable(["dft64"])
        for spec in specs:
            mode, depth, layers = (spec.split(":") + ["", ""])[:3]  # "mode[:depth[:layer mask]]"
            _lib.call("avc_lstm_persist_tune", int(mode))
            if depth:
                _lib.call("avc_lstm_persist_depth", int(depth))
            if layers:
                _lib.call("avc_lstm_persist_layers", int(layers))
            for _ in range(3):
                out = ae(x, co, ct)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            keep = []
            for _ in range(20):
                out = ae(x, co, ct)
                keep.append([o.clone() for o in out])
                if sync_each:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            per = [max((a - b).abs().max().item() for a, b in zip(k, ref)) for k in keep]
            for j in range(len(keep)):
                print(f"  call {j}: max|d| mel/mel_post/codes " +
                      " ".join(f"{(a - b).abs().max().item():.2e}" for a, b in zip(keep[j], ref)), flush=True)
            print("per-call max|d|: " + " ".join(f"{v:.1e}" for v in per), flush=True)
            ms = (time.perf_counter() - t0) / 20 * 1e3
            d = max((a - b).abs().max().item() for a, b in zip(out, ref))
            g = ctypes.c_long(0)
            _lib.call("avc_lstm_persist_status", ctypes.byref(g))
            if not eager_check:
                print(f"modes {spec}: {ms:.3f} ms graph max|d| {d:.2e}; giveups {g.value}", flush=True)
                continue
            cls = [c for c in ("lstm2_persist", "lstm1_persist", "lstm_step_fwd") if c in _lib.TIMING_CLASSES]
            _lib.timing_enable(cls)
            _lib.timing_reset()
            e = ae(x, co, ct)
            torch.cuda.synchronize()
            cnt = {c: _lib.timing_read(c)["launches"] for c in cls}
            _lib.timing_enable([])
            de = max((a - b).abs().max().item() for a, b in zip(e, ref))
            print(f"modes {spec}: {ms:.3f} ms graph max|d| {d:.2e}; eager max|d| {de:.2e} launches {cnt}; "
                  f"giveups {g.value}", flush=True)
        N = 0
    if how == "switch":  # mode 0 block (no host sync), then a mode-2 block compared call by call
        for mode in (0, 2, 0, 2):
            _lib.call("avc_lstm_persist_tune", mode)
            for i in range(12):
                out = ae(x, co, ct)
                if mode == 2:
                    torch.cuda.synchronize()
                    d = max((a - b).abs().max().item() for a, b in zip(out, ref))
                    print(f"switch mode {mode} call {i}: max|d| {d:.2e}", flush=True)
            torch.cuda.synchronize()
            d = max((a - b).abs().max().item() for a, b in zip(out, ref))
            print(f"switch block mode {mode} end: max|d| {d:.2e}", flush=True)
        N = 0
    for i in range(N):
        if how == "bump" and i % 8 == 0:  # same settings, new config epoch: drop + recapture the graph
            _lib.call("avc_lstm_persist_tune", 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = ae(x, co, ct)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        d = max((a - b).abs().max().item() for a, b in zip(out, ref))
        if d != 0:
            bad.append((i, round(ms, 3), d))
        print(f"{how} call {i}: {ms:.3f} ms max|d| {d:.2e}", flush=True)
g = ctypes.c_long(0)
_lib.call("avc_lstm_persist_status", ctypes.byref(g))
print(f"{how}: {len(bad)} of {N} calls differ: {bad[:10]}; giveups {g.value}")
