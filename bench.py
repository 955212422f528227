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
--mode long runs BASELINE config 5: 32 utterances of U{256..1024} frames zero-padded to 1024
(collate_fn), one Generator forward; `value` counts the utterances' own (unpadded) frames.

The SURVEY §8f rows either side of the Generator have their own lines (replicas, like fwd):
--mode mel  the auto-encoder mel frontend (spectrogram.py:62-142) of one 60 s utterance;
--mode se   the speaker encoder's embed_utterance (speaker_encoder/model.py:142-194) of one
            10 s utterance (16 kHz mel, 12 partials through the 3-layer LSTM, mean + L2).
--mode vocoder  the WaveRNN vocoder's generate (wavernn/model.py:214-329) of one 10 s utterance's
            mel: up-sampling, the batched per-sample loop (20 fold rows x 12,100 steps), cross-fade.

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
PEAK_FP64_MATRIX_TFLOPS = 78.6    # AMD MI355X datasheet (fp64 matrix = fp64 vector); not in the guide
# Roofline of each timed kernel class.  Forward and backward contractions run as 3 f16 MFMA
# products per fp32 product, so their fp32-equivalent MFMA ceiling is 2500/3
# TFLOP/s; the LSTM step streams its (split) weights every time step and is priced against HBM;
# the BPTT step (lstm_step_bwd: split-K 3xf16 product + row epilogue) likewise against 2500/3.
ROOFLINE = {
    "fwd": {"gemm": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3), "lstm_step_fwd": ("hbm", PEAK_HBM_GBS),
            "lstm32": ("hbm", PEAK_HBM_GBS), "lstm2_persist": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3),
            "lstm1_persist": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3)},
    "long": {"gemm": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3), "lstm_step_fwd": ("hbm", PEAK_HBM_GBS),
             "lstm32": ("hbm", PEAK_HBM_GBS), "lstm2_persist": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3),
            "lstm1_persist": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3)},
    "train": {"gemm": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3), "lstm_step_fwd": ("hbm", PEAK_HBM_GBS),
              "lstm_step_bwd": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3), "lstm32": ("hbm", PEAK_HBM_GBS),
              "lstm2_persist": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3),
            "lstm1_persist": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3)},
    "mel": {"dft64": ("mfma", PEAK_FP64_MATRIX_TFLOPS), "gemm": ("mfma", PEAK_FP32_MATRIX_TFLOPS)},
    "se": {"lstm_step_fwd": ("hbm", PEAK_HBM_GBS), "gemm": ("mfma", PEAK_F16_MATRIX_TFLOPS / 3),
           "dft64": ("mfma", PEAK_FP64_MATRIX_TFLOPS)},
    # the sample loop re-reads every loop weight (15.1 MB) once per step from the XCD L2s; priced
    # against HBM bandwidth as the streaming ceiling, the loop itself is bound by its 5 dependent
    # launches per step
    "vocoder": {"wavernn": ("hbm", PEAK_HBM_GBS)},
}
MEL_SECONDS, SE_SECONDS, VOC_SECONDS = 60, 10, 10
# fp32 storage and accumulation; contractions as 3 f16 MFMA products of hi/lo-split operands
# (22 significant bits per operand, range-guarded), DESIGN.md §3
DTYPE = "f32 (3xf16 split, fp32 accumulate)"
METRIC = "mel-frames/sec/GPU AutoVC fwd, 80×128 batch; max|Δmel| vs ref"


def parse():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["fwd", "train", "long", "mel", "se", "vocoder"], default="fwd")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 64 fwd / 256 train)")
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound on the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip the per-launch HIP-event timing")
    return ap.parse_args()


def spawn_ranks(args):
    """`bench.py --gpus N` (N > 1) started without torchrun: launch N ranks (one process per GPU)
    under torch.distributed.run as a child process, before anything touches the GPU, and exit with
    its status.  A multi-GPU request is never measured on fewer GPUs than asked for."""
    import socket
    import subprocess
    n = torch.cuda.device_count()  # does not initialise the GPU on this image
    if n < args.gpus:
        raise SystemExit(f"--gpus {args.gpus} requested but only {n} GPU(s) are visible")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    raise SystemExit(subprocess.call(cmd))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from autovc_amd import _lib

    if args.mode in ("fwd", "train"):
        m = setup_generator(args, dev, rank)
    elif args.mode == "long":
        m = setup_long(args, dev, rank)
    elif args.mode == "mel":
        m = setup_mel(args, dev, rank)
    elif args.mode == "vocoder":
        m = setup_vocoder(args, dev, rank)
    else:
        m = setup_se(args, dev, rank)
    step = m["step"]

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

    extra = m["extra"]() if m.get("extra") else {}

    # Roofline region: the same K steps again with every launch of the kernel classes bracketed
    # by HIP events on its stream (the events cost ~7 us per launch, so `value` above is taken
    # from the uninstrumented region).
    classes = m["classes"]
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

    units = world * m["units_per_step"] * args.steps
    value = units / elapsed
    result = {
        "metric": m["metric"],
        "value": round(value, 1),
        "unit": m["unit"],
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": m["dtype"],
        "data": m["data"],
        "config": m["config"](world),
    }
    if m.get("flop_per_unit"):
        result["achieved_tflops_whole_step"] = round(m["flop_per_unit"] * value / world / 1e12, 2)
    result.update(extra)

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
                unit = "TFLOP/s" + (" (fp32-equivalent, 3 f16 products each)" if peak < 1000 and peak > 500 else
                                    " (fp64)" if peak == PEAK_FP64_MATRIX_TFLOPS else "")
            result["roofline"] = {
                "kernel": dom, "bound": bound, "achieved": round(achieved, 2), "peak": round(peak, 1),
                "unit": unit, "frac": round(achieved / peak, 4),
                "traffic": None,
                "avg_launch_us": kern[dom]["avg_us"],
                "flop_per_launch": round(r["flops"] / r["launches"]),
                "algorithmic_bytes_per_launch": round(r["bytes"] / r["launches"]),
            }
            if dom == "dft64":
                # the STFT runs as one fp64 product against a cos/-sin basis: `achieved`
                # counts that product's FLOP, about 40x what an FFT of the same frames needs, so
                # the fraction prices the matrix engine's use, not the transform's efficiency
                result["roofline"]["work"] = "DFT-as-GEMM FLOP (an FFT needs ~1/40 of them)"
            tr = pmc_traffic(dom, args)
            if tr:
                result["roofline"]["traffic"] = tr["traffic_bytes"]
                result["roofline"]["traffic_source"] = tr["source"]
        result["kernels"] = kern
        result["instrumented_ms_per_step"] = round(1000 * inst_elapsed / args.steps, 3)

    if rank == 0 and world == 1 and not args.no_cpu and m.get("cpu"):
        result["cpu_baseline"], extra = m["cpu"](out)
        result.update(extra)
    elif "cpu_baseline" not in result:
        result["cpu_baseline"] = None

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def setup_generator(args, dev, rank):
    """C2 forward (default) or C3/C4 training step of the Generator."""
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

    fwd = args.mode == "fwd"

    def convert_call():
        """The same batch called exactly as VoiceConverter.convert() calls the Generator
        (voice_converter.py:172-174): grad mode on, parameters requiring grad, outputs carrying a
        grad_fn (the fused forward under one recomputing autograd node)."""
        assert all(p.requires_grad for p in model.parameters())
        outs = None
        for _ in range(max(2, args.warmup)):
            outs = model(x, c_org, c_trg)
        assert outs[1].grad_fn is not None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            outs = model(x, c_org, c_trg)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        return {"value": round(B * T / dt, 1), "unit": "mel-frames/s", "ms_per_step": round(1000 * dt, 3)}

    def eval_bn():
        """The same batch with eval-mode BN (running statistics), reported beside the train-mode
        headline ("eval also reported"); and the convert()-style grad-enabled call."""
        conv = convert_call()
        model.eval()
        with torch.no_grad():
            for _ in range(max(2, args.warmup)):  # eager, then graph capture
                model(x, c_org, c_trg)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                model(x, c_org, c_trg)
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        model.train()
        return {"eval_bn": {"value": round(B * T / dt, 1), "unit": "mel-frames/s", "ms_per_step": round(1000 * dt, 3)},
                "convert_call": conv}

    return {
        "step": step, "units_per_step": B * T, "unit": "mel-frames/s", "dtype": DTYPE,
        "metric": METRIC if fwd else "mel-frames/sec AutoVC train step, 80×128 batch",
        "data": "synthetic (U[0,1) mels, |N(0,1)| L2-normalised speaker embeddings; seeded synthetic weights)",
        "classes": ["gemm", "lstm_step_fwd", "lstm32", "lstm2_persist", "lstm1_persist"] + ([] if fwd else ["lstm_step_bwd"]),
        "flop_per_unit": 56.77e6 if fwd else 192.2e6,
        "config": lambda world: {
            "workload": ("C2: batch=64 synthetic 80x128 mels, Generator forward (conversion path, train-mode BN "
                         "as convert() runs), whole-Generator HIP path") if fwd else
                        ("C3/C4: batch=256/GPU training step: fwd + loss (2nd encoder pass) + bwd + "
                         "RCCL all-reduce + fused clip/Adam/EMA"),
            "global_batch": world * B,
            "frames_per_utterance": T,
            "parallelism": (f"replicas x{world}" if fwd else f"dp{world}"),
            "algorithmic_gflop_per_step": round((56.77e6 if fwd else 192.2e6) * B * T / 1e9, 1),
        },
        "cpu": ((lambda out: _with_dmel(cpu_baseline(args, sd, x_np, out, B, T, rank))) if fwd else
                (lambda out: (cpu_train_baseline(args, sd, T, B), {}))),
        "extra": eval_bn if fwd else None,
    }


def setup_long(args, dev, rank):
    """C5 long-form conversion: B = 32 utterances, lengths U{256..1024} (seed 2), zero-padded to
    1024 frames as collate_fn does (dataloader.py:112-121), one fused Generator forward with
    train-mode BN (what convert() runs).  The same batch is the C5 parity case of
    tests/test_gpu_model.py::test_c5_long_form_against_oracle."""
    import numpy as np
    from autovc_amd.auto_encoder import AutoEncoder
    from autovc_amd.weights import synthetic_embedding, synthetic_mel, torch_state_dict

    B = args.batch or 32
    T = 1024 if args.frames == 128 else args.frames
    rng = np.random.default_rng(2 + rank)
    lengths = rng.integers(min(256, T), T + 1, size=B)
    x_np = synthetic_mel(12 + rank, B, T)
    for i, n in enumerate(lengths):
        x_np[i, :, n:] = 0.0
    valid = int(lengths.sum())
    sd = torch_state_dict(0)
    model = AutoEncoder(device=dev, verbose=False)
    model.load_state_dict(sd)
    model.to(dev).train()
    x = torch.from_numpy(x_np).to(dev)
    c_org = torch.from_numpy(synthetic_embedding(112 + rank, B)).to(dev)
    c_trg = torch.from_numpy(synthetic_embedding(212 + rank, B)).to(dev)

    def step():
        with torch.no_grad():
            return model(x, c_org, c_trg)

    def cpu(out):
        from oracle import autovc_oracle as orc
        cores, cpu_desc = _cpu_share()
        torch.set_num_threads(cores)
        # bounded sample: the first 4 utterances of the batch (same lengths, same padding)
        n = min(4, B)
        xs = torch.from_numpy(x_np[:n])
        co, ct = c_org[:n].cpu(), c_trg[:n].cpu()
        bufs = {k: v.clone() for k, v in sd.items() if "running" in k}
        times = []
        with torch.no_grad():
            orc.forward(sd, xs, co, ct, True, bufs)
            t_start = time.perf_counter()
            while len(times) < 2 or (time.perf_counter() - t_start < args.cpu_seconds and len(times) < 10):
                t1 = time.perf_counter()
                orc.forward(sd, xs, co, ct, True, bufs)
                times.append(time.perf_counter() - t1)
        times.sort()
        med = times[len(times) // 2]
        return ({"value": round(float(lengths[:n].sum()) / med, 1), "unit": "mel-frames/s", "cores": cores,
                 "kind": "port",
                 "sample": f"{len(times)} timed reps of the first {n} utterances of the C5 batch (padded to {T}) "
                           f"through the oracle forward, median; unpadded frames counted; "
                           f"{torch.get_num_threads()} torch threads; {cpu_desc}"}, {})

    return {
        "step": step, "units_per_step": valid, "unit": "mel-frames/s", "dtype": DTYPE,
        "metric": "mel-frames/sec AutoVC long-form fwd (C5: ragged lengths <= 1024, zero-padded)",
        "data": "synthetic (U[0,1) mels zero-padded past each length, |N(0,1)| L2-normalised embeddings; "
                "seeded synthetic weights)",
        "classes": ["gemm", "lstm_step_fwd", "lstm32", "lstm2_persist", "lstm1_persist"],
        "flop_per_unit": 56.77e6 * B * T / valid,
        "config": lambda world: {
            "workload": f"C5: batch={B} utterances, lengths U{{256..{T}}} zero-padded to {T} frames, Generator "
                        "forward (train-mode BN), whole-Generator HIP path",
            "global_batch": world * B, "frames_per_utterance": T, "valid_frames_per_step": valid,
            "parallelism": f"replicas x{world}",
            "algorithmic_gflop_per_step": round(56.77e6 * B * T / 1e9, 1)},
        "cpu": cpu,
    }


def _cpu_share():
    """Threads for a CPU baseline: every core of this process's affinity set, except that a box
    which grants this job a share of a larger machine says so in OMP_NUM_THREADS (the GPU boxes
    here: 16 per GPU, of the whole machine's cores) -- the share is then used.  Returns (threads,
    a description naming the CPU model and both counts)."""
    aff = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS", "")
    n = min(aff, int(share)) if share.isdigit() and int(share) > 0 else aff
    model = "unknown CPU"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    why = f" (the job's CPU share, OMP_NUM_THREADS={share})" if n < aff else " (the whole affinity set)"
    return n, f"{n} threads of {aff} in the affinity set{why}, {model}"


def _with_dmel(r):
    return r[0], {"max_abs_dmel_vs_cpu": r[1]}


def setup_mel(args, dev, rank):
    """AE mel frontend (spectrogram.py:62-142) of one 60 s synthetic-speech utterance."""
    from autovc_amd.audio import spectrogram as sp
    from autovc_amd.weights import synthetic_speech

    sr, hop = 22050, 275
    wav_np = synthetic_speech(11 + rank, MEL_SECONDS * sr, sr)
    wav = torch.from_numpy(wav_np).to(dev)
    F = 1 + len(wav_np) // hop

    def step():
        return sp.mel_spec_auto_encoder(wav, device=dev)

    def cpu(out):
        from oracle import audio_oracle as ao
        ao.mel_spec_auto_encoder(wav_np[: sr * 5])  # warm
        times = []
        t_start = time.perf_counter()
        while len(times) < 2 or (time.perf_counter() - t_start < args.cpu_seconds and len(times) < 20):
            t1 = time.perf_counter()
            ref = ao.mel_spec_auto_encoder(wav_np)
            times.append(time.perf_counter() - t1)
        times.sort()
        med = times[len(times) // 2]
        d = float((out.float().cpu() - ref).abs().max())
        _, cpu_desc = _cpu_share()
        return ({"value": round(F / med, 1), "unit": "mel-frames/s", "cores": 1, "kind": "port",
                 "sample": f"{len(times)} timed reps of the same 60 s utterance through the float64 numpy "
                           f"restatement (oracle/audio_oracle.py; numpy rfft, single thread: numpy's FFT "
                           f"does not thread), median; CPU: {cpu_desc}"},
                {"max_abs_dmel_vs_cpu": d})

    return {
        "step": step, "units_per_step": F, "unit": "mel-frames/s", "dtype": "f64 DFT / f32 mel",
        "metric": "mel-frames/sec AE mel frontend (|STFT| n_fft 2048 hop 275 win 1100 -> 80 mels -> dB-normalised)",
        "data": "synthetic speech-like waveform (autovc_amd.weights.synthetic_speech), 22.05 kHz",
        "classes": ["dft64", "gemm"], "flop_per_unit": 2.0 * 2 * 1025 * 1100 + 2.0 * 1028 * 80,
        "config": lambda world: {"workload": f"one {MEL_SECONDS} s utterance per GPU ({F} frames), "
                                             "mel_spec_auto_encoder", "global_batch": world,
                                 "frames_per_utterance": F, "parallelism": f"replicas x{world}"},
        "cpu": cpu,
    }


def setup_se(args, dev, rank):
    """Speaker encoder embed_utterance (speaker_encoder/model.py:142-194) of one 10 s utterance."""
    from autovc_amd.speaker_encoder import SpeakerEncoder
    from autovc_amd.weights import speaker_encoder_state_dict, synthetic_speech

    sr = 16000
    sd = speaker_encoder_state_dict(0)
    se = SpeakerEncoder(device=dev, verbose=False)
    se.load_state_dict(sd)
    wav_np = synthetic_speech(21 + rank, SE_SECONDS * sr, sr)

    def step():
        return se.embed_utterance(wav_np)

    def cpu(out):
        from oracle import audio_oracle as ao
        cores, cpu_desc = _cpu_share()
        torch.set_num_threads(cores)
        ref = ao.embed_utterance(sd, wav_np)
        times = []
        t_start = time.perf_counter()
        while len(times) < 2 or (time.perf_counter() - t_start < args.cpu_seconds and len(times) < 20):
            t1 = time.perf_counter()
            ao.embed_utterance(sd, wav_np)
            times.append(time.perf_counter() - t1)
        times.sort()
        med = times[len(times) // 2]
        d = float(abs(out.numpy() - ref).max())
        return ({"value": round(SE_SECONDS / med, 2), "unit": "audio-seconds/s", "cores": cores, "kind": "port",
                 "sample": f"{len(times)} timed reps of the same 10 s utterance through the oracle (numpy float64 "
                           f"mel + torch-CPU LSTM, {torch.get_num_threads()} threads), median; {cpu_desc}"},
                {"max_abs_dembed_vs_cpu": d})

    return {
        "step": step, "units_per_step": SE_SECONDS, "unit": "audio-seconds/s", "dtype": "f32 (f64 DFT)",
        "metric": "audio-seconds/sec speaker-encoder embed_utterance (16 kHz, 160-frame partials, 3x256 LSTM)",
        "data": "synthetic speech-like waveform, 16 kHz; seeded synthetic weights",
        "classes": ["lstm_step_fwd", "gemm", "dft64"],
        "config": lambda world: {"workload": f"one {SE_SECONDS} s utterance per GPU per step (12 partials x 160 "
                                             "frames), embed_utterance incl. its mel frontend",
                                 "global_batch": world, "parallelism": f"replicas x{world}"},
        "cpu": cpu,
    }


def setup_vocoder(args, dev, rank):
    """WaveRNN generate (wavernn/model.py:214-329) of one 10 s utterance's 80-mel (802 frames):
    batched fold (target 11,000, overlap 550) -> 20 rows x 12,100 sequential sample steps."""
    from autovc_amd.wavernn import WaveRNN
    from autovc_amd.weights import synthetic_mel, wavernn_state_dict

    sr, hop = 22050, 275
    T = VOC_SECONDS * sr // hop
    sd = wavernn_state_dict(0)
    net = WaveRNN(device=dev)
    net.load_state_dict(sd)
    mel_np = synthetic_mel(31 + rank, 1, T)
    mel = torch.from_numpy(mel_np).to(dev)
    audio_s = (T - 1) * hop / sr

    def step():
        return net.generate(mel)

    def cpu(out):
        from oracle import wavernn_oracle as wo
        cores, cpu_desc = _cpu_share()
        torch.set_num_threads(cores)
        n = 60
        wo.generate(sd, torch.from_numpy(mel_np), steps=4)  # warm
        t1 = time.perf_counter()
        part = wo.generate(sd, torch.from_numpy(mel_np), steps=n)
        dt = time.perf_counter() - t1
        L = 11_000 + 2 * 550
        per_call = dt / n * L
        return ({"value": round(audio_s / per_call, 3), "unit": "audio-seconds/s", "cores": cores, "kind": "port",
                 "sample": f"the first {n} of the {L} sequential steps (all {part.shape[0]} fold rows) of the same "
                           f"generate() through the oracle (torch-CPU, {torch.get_num_threads()} threads), "
                           f"extrapolated linearly to the whole loop (every step is the same work); {cpu_desc}"},
                {"fold_rows": int(part.shape[0]), "sequential_steps": L})

    return {
        "step": step, "units_per_step": audio_s, "unit": "audio-seconds/s", "dtype": "f32",
        "metric": "audio-seconds/sec WaveRNN generate (MOL, batched: target 11000, overlap 550)",
        "data": "synthetic U[0,1) 80-mel of a 10 s utterance; seeded synthetic weights (no checkpoint offline)",
        "classes": ["wavernn"],
        "config": lambda world: {"workload": f"one {VOC_SECONDS} s utterance per GPU ({T} mel frames -> "
                                             f"{(T - 1) * hop} samples), WaveRNN.generate incl. up-sampling and "
                                             "cross-fade", "global_batch": world, "parallelism": f"replicas x{world}"},
        "cpu": cpu,
    }


def pmc_traffic(cls, args):
    """HBM bytes per launch of kernel class `cls` (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected)
    from the newest committed rocprofv3 PMC summary of this same default command
    (profiles/rNN_pmc_traffic.json, written by scripts/pmc_traffic.py); counters cannot be read
    from inside the process, so the number is the profiled run's, not this run's."""
    import glob
    # default commands only: C2 forward (profiles/rNN_pmc_traffic.json), C3 training step
    # (profiles/rNN_pmc_traffic_train.json), C5 long-form forward (profiles/rNN_pmc_traffic_long.json)
    if args.frames != 128 or args.mode not in ("fwd", "train", "long"):
        return None
    if args.batch not in (None, {"fwd": 64, "train": 256, "long": 32}[args.mode]):
        return None
    pat = {"fwd": "r*_pmc_traffic.json", "train": "r*_pmc_traffic_train.json",
           "long": "r*_pmc_traffic_long.json"}[args.mode]
    files = sorted(glob.glob(os.path.join(HERE, "profiles", pat)))
    if not files:
        return None
    with open(files[-1]) as fh:
        c = json.load(fh)["classes"].get(cls)
    if not c:
        return None
    return {"traffic_bytes": c["traffic_bytes"], "source": os.path.relpath(files[-1], HERE)}


def cpu_train_baseline(args, sd, T, B=256):
    """Oracle training step (oracle/autovc_oracle.py Trainer: fwd, _loss with the second encoder
    pass, autograd backward, clip 1.0, Adam, EMA -- model.py:303-321) on this host's cores, at the
    bench's own batch (B = 256: ~6 s per step on 16 threads): one warm step, then timed steps until
    --cpu-seconds have passed (at least one)."""
    from oracle import autovc_oracle as orc
    from autovc_amd.weights import onehot_embedding, synthetic_mel
    cores, cpu_desc = _cpu_share()
    torch.set_num_threads(cores)
    X = torch.from_numpy(synthetic_mel(1, B, T))
    c = torch.from_numpy(onehot_embedding(B))
    tr = orc.Trainer(sd)
    tr.step(X, c)  # warm
    times = []
    t_start = time.perf_counter()
    while not times or (time.perf_counter() - t_start < args.cpu_seconds and len(times) < 10):
        t1 = time.perf_counter()
        tr.step(X, c)
        times.append(time.perf_counter() - t1)
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(B * T / med, 1), "unit": "mel-frames/s", "cores": cores, "kind": "port",
            "sample": f"{len(times)} timed training steps (+1 warm) of the bench's B={B}, T={T} one-hot batch "
                      f"through the oracle Trainer, median; {torch.get_num_threads()} torch threads; {cpu_desc}"}


def cpu_baseline(args, sd, x_np, gpu_out, B, T, rank):
    """Oracle forward (torch-CPU restatement, `port`) on this host's cores, same batch."""
    from oracle import autovc_oracle as orc
    from autovc_amd.weights import synthetic_embedding
    cores, cpu_desc = _cpu_share()
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
                       f"forward, median; {torch.get_num_threads()} torch threads; {cpu_desc}"}, dmel)


if __name__ == "__main__":
    main()
