# C2 forward + C3 step A/B of the library named by $1 (default ablib/prev.so) against the in-tree
# build: alternating processes, three rounds; then bit-identity of the two builds' C2 outputs
set -e
prev=${1:-ablib/prev.so}
for i in 1 2 3; do
  AUTOVC_HIP_LIB=$prev timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu >> gpurun_out/abf_prev.log 2>&1
  timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu >> gpurun_out/abf_new.log 2>&1
done
python - <<'PY'
import json
for n in ("prev", "new"):
    v = [json.loads(l)["ms_per_step"] for l in open(f"gpurun_out/abf_{n}.log") if l.startswith("{")]
    print(n, "C2 ms/step", v)
PY
AUTOVC_HIP_LIB=$prev timeout -k 10 120 python scripts/compare_libs.py gpurun_out/cmp_prev.pt
timeout -k 10 120 python scripts/compare_libs.py gpurun_out/cmp_new.pt
python scripts/compare_libs.py --diff gpurun_out/cmp_prev.pt gpurun_out/cmp_new.pt
for i in 1 2; do
  AUTOVC_HIP_LIB=$prev timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abt_prev.log 2>&1
  timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abt_new.log 2>&1
done
grep -H median gpurun_out/abt_prev.log gpurun_out/abt_new.log
