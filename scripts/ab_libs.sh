# C3 step time of several library builds (arguments), alternating processes, two rounds
set -e
for i in 1 2; do
  for lib in "$@"; do
    AUTOVC_HIP_LIB=$lib timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abl.log 2>&1
  done
done
grep median gpurun_out/abl.log
