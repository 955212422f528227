# A/B of the C3 step time: the library named by $1 (default ablib/prev.so) against the in-tree
# build, alternating processes, two rounds each
set -e
prev=${1:-ablib/prev.so}
for i in 1 2; do
  AUTOVC_HIP_LIB=$prev timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abt.log 2>&1
  timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abt.log 2>&1
done
grep median gpurun_out/abt.log
