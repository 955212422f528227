# Same-box A/B of a saved library (argv[1], default ab/r05.so = the driver-benched round-5 build) against the in-tree
# build: C2 forward and C5 long-form batch, alternating processes, three rounds each.
set -e
lib=${1:-ab/r05.so}; tag=$(basename $lib .so)
mkdir -p gpurun_out
rm -f gpurun_out/ab5_*.log
for i in 1 2 3; do
  AUTOVC_WGRAD_IMAGE=${REF_WGRAD:-0} AUTOVC_HIP_LIB=$lib timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu >> gpurun_out/ab5_c2_$tag.log 2>&1
  timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-cpu >> gpurun_out/ab5_c2_new.log 2>&1
done
for i in 1 2 3; do
  AUTOVC_WGRAD_IMAGE=${REF_WGRAD:-0} AUTOVC_HIP_LIB=$lib timeout -k 10 150 python bench.py --mode long --steps 8 --warmup 2 --no-cpu >> gpurun_out/ab5_c5_$tag.log 2>&1
  timeout -k 10 150 python bench.py --mode long --steps 8 --warmup 2 --no-cpu >> gpurun_out/ab5_c5_new.log 2>&1
done
for f in c2_$tag c2_new c5_$tag c5_new; do
  python -c "
import json,sys
L=[json.loads(x) for x in open(sys.argv[2]) if x.startswith('{')]
print(sys.argv[1], 'ms/step', [d['ms_per_step'] for d in L], 'lstm2 us', [round(d.get('kernels',{}).get('lstm2_persist',{}).get('avg_us',0),1) for d in L], 'lstm1 us', [round(d.get('kernels',{}).get('lstm1_persist',{}).get('avg_us',0),1) for d in L], 'gemm us', [round(d.get('kernels',{}).get('gemm',{}).get('avg_us',0),1) for d in L])" $f gpurun_out/ab5_$f.log
done
