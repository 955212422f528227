set -e
for i in 1 2 3; do
  for lib in ablib/prev.so ablib/cap256.so autovc_amd/libautovc_hip.so; do
    AUTOVC_HIP_LIB=$lib timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu | sed "s|^|$lib |" >> gpurun_out/ab3f.log 2>&1
  done
done
for i in 1 2; do
  for lib in ablib/prev.so ablib/cap256.so autovc_amd/libautovc_hip.so; do
    AUTOVC_HIP_LIB=$lib timeout -k 10 120 python scripts/train_time.py >> gpurun_out/ab3t.log 2>&1
  done
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab3f.log"):
    lib, _, js = l.partition(" ")
    if js.startswith("{"): d[lib].append(json.loads(js)["ms_per_step"])
for k, v in d.items(): print("C2", k, v)
PY
grep median gpurun_out/ab3t.log
