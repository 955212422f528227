# Same-box A/B of the round-5 library (ab/r05.so, the driver-benched build) against the in-tree
# build: C2 forward and C5 long-form batch, alternating processes, three rounds each.
set -e
mkdir -p gpurun_out
rm -f gpurun_out/ab5_*.log
for i in 1 2 3; do
  AUTOVC_HIP_LIB=ab/r05.so timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu >> gpurun_out/ab5_c2_r05.log 2>&1
  timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu >> gpurun_out/ab5_c2_new.log 2>&1
done
for i in 1 2 3; do
  AUTOVC_HIP_LIB=ab/r05.so timeout -k 10 150 python bench.py --mode long --steps 8 --warmup 2 --no-timing --no-cpu >> gpurun_out/ab5_c5_r05.log 2>&1
  timeout -k 10 150 python bench.py --mode long --steps 8 --warmup 2 --no-timing --no-cpu >> gpurun_out/ab5_c5_new.log 2>&1
done
for f in c2_r05 c2_new c5_r05 c5_new; do
  python -c "import json,sys; print(sys.argv[1], 'ms/step', [json.loads(x)['ms_per_step'] for x in open(sys.argv[2]) if x.startswith('{')])" $f gpurun_out/ab5_$f.log
done
