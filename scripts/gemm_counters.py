#!/usr/bin/env python3
"""Summarise the `gpu_check.sh gpmc` passes (rocprofv3 --pmc on scripts/gemm_micro.py) for the
split-f16 GEMM: MFMA busy fraction, wait fractions and L2 hit rate per kernel shape.

Usage: gemm_counters.py GPMC_DIR OUT.json

SQ_*_CYCLES / SQ_WAIT_* count in quad-cycles except SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed
over SIMDs); MFMA busy fraction = MFMA_BUSY / (SIMDs x kernel cycles), kernel cycles from
SQ_BUSY_CYCLES / (shader engines) — both as read on gfx950 (MI355X: 1024 SIMDs, 32 SEs).
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    d, out = sys.argv[1:3]
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        # pass directories are named <mode>_<first counter> (gpu_check.sh gpmc3): the mode of
        # gemm_micro.py that ran (c2 / c3fwd / c3bwd)
        mode = next((m for m in ("c3fwd", "c3bwd", "c2") if f"/{m}_" in f), "")
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "gemm16f" not in n:
                continue
            g = r.get("Grid_Size", "")
            shape = {("c2", "131072"): "conv 512->512 k5 fwd, M=8192 N=512 K=2560",
                     ("", "131072"): "conv 512->512 k5 fwd, M=8192 N=512 K=2560",
                     ("c2", "1048576"): "lstm2 input projection, M=8192 N=4096 K=512",
                     ("", "1048576"): "lstm2 input projection, M=8192 N=4096 K=512",
                     ("c3fwd", "524288"): "conv 512->512 k5 fwd, M=32768 N=512 K=2560",
                     ("c3bwd", "524288"): "conv 512->512 k5 dgrad (5 of 6 launches; 1 fwd), M=32768 N=512 K=2560",
                     }.get((mode, g), "wgrad (split-K / tap-batched)" if mode == "c3bwd" else "")
            key = f"{mode} gemm16f grid={g} {shape}".strip()
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, c in vals.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        cyc = m["SQ_BUSY_CYCLES"] / 32.0
        res[k] = {
            "counters": {n: round(v) for n, v in m.items()},
            "kernel_cycles_est": round(cyc),
            "mfma_busy_frac": round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 3),
            "wait_inst_frac_of_wave_cycles": round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3),
            "l2_hit_rate": round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 3),
        }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: {x: v[x] for x in v if x != "counters"} for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
