"""Operand-prep share of one C3 step from a rocprofv3 kernel trace (gpu_check.sh ktrain): the
kernels of the step between the two Adam launches, grouped; prep = split_frag32*, split_convw,
absmax_vec, guard_scan."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ktrain/train_kernel_trace.csv")))
idx = [i for i, r in enumerate(rows) if "adam_ema" in r["Kernel_Name"]]
st = rows[idx[0] + 1:idx[1] + 1]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(dur(r) for r in st)
g = defaultdict(lambda: [0, 0.0])
for r in st:
    n = r["Kernel_Name"]
    for k in ("split_frag32_dual", "split_frag32", "split_convw", "absmax_vec", "guard_scan", "gemm16f", "bptt", "lstm_persist"):
        if k in n:
            n = k
            break
    g[n][0] += 1
    g[n][1] += dur(r)
prep = sum(v[1] for k, v in g.items() if k in ("split_frag32_dual", "split_frag32", "split_convw", "absmax_vec", "guard_scan"))
print(f"step kernels {len(st)}, busy {tot:.0f} us; operand prep {prep:.0f} us = {100 * prep / tot:.2f} %")
for k, (c, d) in sorted(g.items(), key=lambda kv: -kv[1][1])[:14]:
    print(f"  {k[:60]:60s} {c:4d} x {d / c:8.1f} us = {d:8.1f} us ({100 * d / tot:5.2f} %)")
