# C2 forward A/B of libraries (default ablib/prev.so) against the in-tree build: alternating
# processes, four rounds, headline ms/step of each
set -e
libs=${@:-ablib/prev.so}
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for l in $libs; do
    AUTOVC_HIP_LIB=$l timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu >> gpurun_out/abc_$(basename $l .so).log 2>&1
  done
  timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu >> gpurun_out/abc_new.log 2>&1
done
for l in $libs new; do
  python -c "import json,sys; print(sys.argv[1], 'C2 ms/step', [json.loads(x)['ms_per_step'] for x in open(sys.argv[2]) if x.startswith('{')])" $l gpurun_out/abc_$(basename $l .so).log
done
