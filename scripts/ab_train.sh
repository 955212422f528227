set -e
for i in 1 2; do
  AUTOVC_HIP_LIB=ablib/prev.so timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abt.log 2>&1
  timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abt.log 2>&1
done
cat gpurun_out/abt.log | grep median
