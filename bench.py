#!/usr/bin/env python3
"""AutoVC Generator throughput on MI355X (BASELINE.json metric).

Default workload = BASELINE config 2: batch 64 of synthetic 80x128 mels through the Generator
forward with train-mode BatchNorm — what VoiceConverter.convert() runs (the reference never calls
.eval()) — on the whole-Generator HIP path.  One "step" = one forward of one batch,
inputs already resident in HBM.  With --gpus N (torchrun, one process per GPU) every rank runs an
independent replica on its own batch: conversion shards by utterance with no collective, so
scaling is "weak" and `value` = all frames of all ranks / max-over-ranks time.

--mode train runs BASELINE config 3/4 instead (batch 256 training step: forward, loss with the
second encoder pass, backward, RCCL gradient all-reduce when N>1, fused clip+Adam+EMA).

Also reported on the same line: `roofline` for the dominant kernel class, measured with HIP
events around every launch of that class inside the timed region, and `cpu_baseline`: the CPU
oracle (oracle/autovc_oracle.py, a torch-CPU restatement pinned to the reference's outputs) timed
on this host's cores on a bounded sample of the same workload (rank 0, N=1 only), together with
max|d mel| of the GPU output against it on the same batch.
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_FP32_MATRIX_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_*_f32, dense
PEAK_F16_MATRIX_TFLOPS = 2500.0   # dense f16/bf16 MFMA
PEAK_HBM_GBS = 8000.0
# Roofline of each timed kernel class.  Forward contractions run as 3 f16 MFMA products per
# fp32 product, so their fp32-equivalent MFMA ceiling is 2500/3 TFLOP/s; the LSTM step streams
# its (split) weights every time step and is priced against HBM; backward products are fp32.
ROOFLINE = {
    "fwd": {"gemm": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3), "lstm_step_fwd": ("hbm", PEAK_HBM_GBS),
            "lstm32": ("hbm", PEAK_HBM_GBS)},
    "train": {"gemm": ("mfma", PEAK_FP32_MATRIX_TFLOPS), "lstm_step_fwd": ("hbm", PEAK_HBM_GBS),
              "lstm_step_bwd": ("mfma", PEAK_FP32_MATRIX_TFLOPS), "lstm32": ("hbm", PEAK_HBM_GBS)},
}
METRIC = "mel-frames/sec/GPU AutoVC fwd, 80×128 batch; max|Δmel| vs ref"


def parse():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["fwd", "train"], default="fwd")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 64 fwd / 256 train)")
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound on the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the per-launch HIP-event timing")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from autovc_amd import _lib
    from autovc_amd.auto_encoder import AutoEncoder
    from autovc_amd.weights import onehot_embedding, synthetic_embedding, synthetic_mel, torch_state_dict

    B = args.batch or (64 if args.mode == "fwd" else 256)
    T = args.frames
    sd = torch_state_dict(0)
    model = AutoEncoder(device=dev, verbose=False)
    model.load_state_dict(sd)
    model.to(dev).train()
    x_np = synthetic_mel(1 + rank, B, T)
    x = torch.from_numpy(x_np).to(dev)
    if args.mode == "fwd":
        c_org = torch.from_numpy(synthetic_embedding(101 + rank, B)).to(dev)
        c_trg = torch.from_numpy(synthetic_embedding(201 + rank, B)).to(dev)

        def step():
            with torch.no_grad():
                return model(x, c_org, c_trg)
    else:
        c = torch.from_numpy(onehot_embedding(B, offset=rank)).to(dev)
        model.configure_optimizer()

        def step():
            return model.train_step(x, c)

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Roofline region: the same K steps again with every launch of the kernel classes bracketed
    # by HIP events on its stream (the events cost ~7 us per launch, so `value` above is taken
    # from the uninstrumented region).
    classes = ["gemm", "lstm_step_fwd", "lstm32"] + (["lstm_step_bwd"] if args.mode == "train" else [])
    inst_elapsed = None
    if not args.no_timing:
        _lib.timing_enable(classes)
        _lib.timing_reset()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        inst_elapsed = time.perf_counter() - t1
        _lib.timing_enable([])

    frames = world * B * T * args.steps
    value = frames / elapsed
    fwd_flop_per_frame = 56.77e6
    result = {
        "metric": METRIC if args.mode == "fwd" else "mel-frames/sec AutoVC train step, 80×128 batch",
        "value": round(value, 1),
        "unit": "mel-frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (U[0,1) mels, |N(0,1)| L2-normalised speaker embeddings; seeded synthetic weights)",
        "config": {
            "workload": ("C2: batch=64 synthetic 80x128 mels, Generator forward (conversion path, train-mode BN "
                         "as convert() runs), whole-Generator HIP path") if args.mode == "fwd" else
                        ("C3/C4: batch=256/GPU training step: fwd + loss (2nd encoder pass) + bwd + "
                         "RCCL all-reduce + fused clip/Adam/EMA"),
            "global_batch": world * B,
            "frames_per_utterance": T,
            "parallelism": (f"replicas x{world}" if args.mode == "fwd" else f"dp{world}"),
            "algorithmic_gflop_per_step": round((fwd_flop_per_frame if args.mode == "fwd" else 192.2e6) * B * T / 1e9, 1),
        },
        "achieved_tflops_whole_step": round((fwd_flop_per_frame if args.mode == "fwd" else 192.2e6) * value / world / 1e12, 2),
    }

    if not args.no_timing:
        per = {c: _lib.timing_read(c) for c in classes}
        kern = {}
        for c, r in per.items():
            if r["launches"] == 0 or r["ms"] <= 0:
                continue
            kern[c] = {"launches_per_step": r["launches"] / args.steps, "avg_us": round(1000 * r["ms"] / r["launches"], 2),
                       "share_of_step": round(r["ms"] / (1000 * inst_elapsed), 3),
                       "tflops": round(r["flops"] / (r["ms"] * 1e-3) / 1e12, 2),
                       "gbs_weights": round(r["bytes"] / (r["ms"] * 1e-3) / 1e9, 1)}
        dom = max(kern, key=lambda c: per[c]["ms"]) if kern else None
        if dom:
            r = per[dom]
            bound, peak = ROOFLINE[args.mode][dom]
            if bound == "hbm":
                achieved = r["bytes"] / (r["ms"] * 1e-3) / 1e9
                unit = "GB/s"
            else:
                achieved = r["flops"] / (r["ms"] * 1e-3) / 1e12
                unit = "TFLOP/s" + (" (fp32-equivalent, 3 f16 products each)" if peak < 1000 and peak > 500 else "")
            result["roofline"] = {
                "kernel": dom, "bound": bound, "achieved": round(achieved, 2), "peak": round(peak, 1),
                "unit": unit, "frac": round(achieved / peak, 4),
                "traffic": None,
                "avg_launch_us": kern[dom]["avg_us"],
                "flop_per_launch": round(r["flops"] / r["launches"]),
                "algorithmic_bytes_per_launch": round(r["bytes"] / r["launches"]),
            }
            tr = pmc_traffic(dom, args)
            if tr:
                result["roofline"]["traffic"] = tr["traffic_bytes"]
                result["roofline"]["traffic_source"] = tr["source"]
        result["kernels"] = kern
        result["instrumented_ms_per_step"] = round(1000 * inst_elapsed / args.steps, 3)

    if rank == 0 and world == 1 and not args.no_cpu and args.mode == "fwd":
        result["cpu_baseline"], result["max_abs_dmel_vs_cpu"] = cpu_baseline(args, sd, x_np, out, B, T, rank)
    elif "cpu_baseline" not in result:
        result["cpu_baseline"] = None

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def pmc_traffic(cls, args):
    """HBM bytes per launch of kernel class `cls` (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected)
    from the newest committed rocprofv3 PMC summary of this same default command
    (profiles/rNN_pmc_traffic.json, written by scripts/pmc_traffic.py); counters cannot be read
    from inside the process, so the number is the profiled run's, not this run's."""
    import glob
    if args.mode != "fwd" or args.batch not in (None, 64) or args.frames != 128:
        return None
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None
    with open(files[-1]) as fh:
        c = json.load(fh)["classes"].get(cls)
    if not c:
        return None
    return {"traffic_bytes": c["traffic_bytes"], "source": os.path.relpath(files[-1], HERE)}


def cpu_baseline(args, sd, x_np, gpu_out, B, T, rank):
    """Oracle forward (torch-CPU restatement, `port`) on this host's cores, same batch."""
    from oracle import autovc_oracle as orc
    from autovc_amd.weights import synthetic_embedding
    cores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    x = torch.from_numpy(x_np)
    c_org = torch.from_numpy(synthetic_embedding(101 + rank, B))
    c_trg = torch.from_numpy(synthetic_embedding(201 + rank, B))
    bufs = {k: v.clone() for k, v in sd.items() if "running" in k}
    with torch.no_grad():
        t0 = time.perf_counter()
        ref = orc.forward(sd, x, c_org, c_trg, True, bufs)  # warm rep
        times = []
        t_start = time.perf_counter()
        while len(times) < 2 or (time.perf_counter() - t_start < args.cpu_seconds and len(times) < 20):
            t1 = time.perf_counter()
            orc.forward(sd, x, c_org, c_trg, True, bufs)
            times.append(time.perf_counter() - t1)
    times.sort()
    med = times[len(times) // 2]
    dmel = float((gpu_out[1].float().cpu() - ref[1]).abs().max())
    return ({"value": round(B * T / med, 1), "unit": "mel-frames/s", "cores": cores, "kind": "port",
             "sample": f"{len(times)} timed reps (+1 warm) of the C2 batch (B={B}, T={T}) through the oracle "
                       f"forward, median; {torch.get_num_threads()} torch threads"}, dmel)


if __name__ == "__main__":
    main()
