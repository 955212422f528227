"""Per-dispatch timeline of the last forward in a rocprofv3 kernel trace (kernel_trace.csv):
start offset, duration and grid of every kernel from the last frames_from_mel launch on."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "frames_from_mel"
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(first)]
seg = rows[idx[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][-50:]
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {name} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}")
print("span", (int(seg[-1]["End_Timestamp"]) - t0) / 1e3, "us")
