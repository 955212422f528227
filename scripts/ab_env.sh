# A/B of the C3 step time between two values of one environment variable ($1 = NAME, $2 = A,
# $3 = B), alternating processes, two rounds each
set -e
for i in 1 2; do
  env "$1=$2" timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abe.log 2>&1 && echo "$1=$2" >> gpurun_out/abe.log
  env "$1=$3" timeout -k 10 120 python scripts/train_time.py >> gpurun_out/abe.log 2>&1 && echo "$1=$3" >> gpurun_out/abe.log
done
grep -A1 median gpurun_out/abe.log
