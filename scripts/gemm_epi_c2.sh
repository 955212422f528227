# The C2 forward (bench.py, per-class kernel timing) against GEMM diagnostic builds: how much of
# the GEMM class is its epilogue (abd_ne: every epilogue skipped, sums kept live; wrong outputs).
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for d in "" ${EPI_DIRS:-abd_ne}; do
    if [ -n "$d" ]; then export AUTOVC_HIP_LIB=$PWD/$d/libautovc_hip.so; else unset AUTOVC_HIP_LIB; fi
    timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | python -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][0]); k=d['kernels']
print('${d:-default}', d['ms_per_step'], 'ms;', ', '.join(f'{c} {v[\"launches_per_step\"]:.0f}x{v[\"avg_us\"]:.1f}us' for c,v in k.items()))"
  done
done
