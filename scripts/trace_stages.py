"""Summarise one forward from a rocprofv3 kernel trace: per-stage busy time and gaps."""
import csv
import sys
from collections import OrderedDict

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if r["Kernel_Name"] != "__amd_rocclr_copyBuffer"]
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
# a forward starts at frames_from_mel_kernel; take the last complete one
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"] == "frames_from_mel_kernel"]
i0 = starts[-2]
i1 = starts[-1]
fw = rows[i0:i1]
span = fw[-1]["e"] - fw[0]["s"]
busy = sum(r["e"] - r["s"] for r in fw)
print(f"kernels {len(fw)}  span {span/1e3:.1f} us  busy {busy/1e3:.1f} us  gaps {(span-busy)/1e3:.1f} us")
# stages: split at lstm32 / lstm_step / gemm boundaries by name runs
stages = OrderedDict()
cur = None
for r in fw:
    n = r["Kernel_Name"]
    key = n
    stages.setdefault(key, [0, 0])
    stages[key][0] += 1
    stages[key][1] += r["e"] - r["s"]
for k, (c, t) in sorted(stages.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:32s} calls {c:4d}  total {t/1e3:8.1f} us  avg {t/c/1e3:7.2f} us")
# lstm step kernels by grid (H=512 vs 1024)
by = {}
for r in fw:
    if r["Kernel_Name"] == "lstm_step_kernel":
        g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Workgroup_Size_X"])
        by.setdefault(g, []).append(r["e"] - r["s"])
for g, v in sorted(by.items()):
    print("lstm_step grid", g, "n", len(v), "avg us", round(sum(v) / len(v) / 1e3, 2), "min", min(v) / 1e3)
gs = [(r["Grid_Size_X"], r["Grid_Size_Y"], (r["e"] - r["s"]) / 1e3) for r in fw if r["Kernel_Name"] == "gemm_kernel"]
print("gemm launches (gridX, gridY, us):", gs)
# gaps between consecutive lstm_step launches
gaps = [fw[i + 1]["s"] - fw[i]["e"] for i in range(len(fw) - 1) if fw[i]["Kernel_Name"] == "lstm_step_kernel" and fw[i + 1]["Kernel_Name"] == "lstm_step_kernel"]
print("gap between lstm steps: avg us", round(sum(gaps) / len(gaps) / 1e3, 2))
