# Effective shader clock of the C2 conv GEMM (gemm_micro.py c2) for the default build and the
# no-load / no-MFMA diagnostic builds: GRBM_GUI_ACTIVE / 8 XCDs / kernel duration
# (MI355X_MICROARCH.md, DVFS give-back).  Writes gpurun_out/gclock_<lib>/.
set -e
for d in "" abd_nl abd_nm; do
  n=${d:-default}
  if [ -n "$d" ]; then export AUTOVC_HIP_LIB=$PWD/$d/libautovc_hip.so; else unset AUTOVC_HIP_LIB; fi
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/gclock_$n -o g -- python3 scripts/gemm_micro.py c2 > gpurun_out/gclock_$n.log 2>&1
done
python3 - <<'PY'
import csv, glob
for n in ("default", "abd_nl", "abd_nm"):
    cc = glob.glob(f"gpurun_out/gclock_{n}/**/*counter_collection.csv", recursive=True)
    kt = glob.glob(f"gpurun_out/gclock_{n}/**/*kernel_trace.csv", recursive=True)
    act = {}
    for f in cc:
        for r in csv.DictReader(open(f)):
            if "gemm16f" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                act.setdefault(r["Grid_Size"], []).append(float(r["Counter_Value"]))
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            if "gemm16f" in r["Kernel_Name"]:
                g = str(int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
                dur.setdefault(g, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for g in act:
        a = sorted(act[g])[len(act[g]) // 2]
        ds = dur.get(g) or dur.get(str(int(g)))
        d = sorted(ds)[len(ds) // 2] if ds else float("nan")
        print(f"{n:8s} grid {g:>8s}: GRBM_GUI_ACTIVE {a:.0f}, kernel {d / 1e3:.1f} us (trace run), clock ~{a / 8 / d:.2f} GHz")
PY
