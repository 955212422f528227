# Same-box A/B of the round-4 tree (ab/r04: its package, .so and bench, copied from the round-4
# commit) against the in-tree build, alternating processes: C2 forward and C5 long-form bench
# lines (three rounds each), C3 step time (two rounds each)
set -e
mkdir -p gpurun_out
unset AUTOVC_HIP_LIB
for i in 1 2 3; do
  (cd ab/r04 && timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu) >> gpurun_out/abtree_r04.log 2>&1
  timeout -k 10 150 python bench.py --steps 30 --warmup 3 --no-timing --no-cpu >> gpurun_out/abtree_new.log 2>&1
  (cd ab/r04 && timeout -k 10 150 python bench.py --mode long --steps 5 --warmup 2 --no-timing --no-cpu) >> gpurun_out/abtree_r04_long.log 2>&1
  timeout -k 10 150 python bench.py --mode long --steps 5 --warmup 2 --no-timing --no-cpu >> gpurun_out/abtree_new_long.log 2>&1
done
for i in 1 2; do
  (cd ab/r04 && timeout -k 10 150 python scripts/train_time.py) >> gpurun_out/abtree_r04_train.log 2>&1
  timeout -k 10 150 python scripts/train_time.py >> gpurun_out/abtree_new_train.log 2>&1
done
for f in r04 new r04_long new_long; do
  python -c "import json,sys; print(sys.argv[1], 'ms/step', [json.loads(x)['ms_per_step'] for x in open(sys.argv[2]) if x.startswith('{')])" $f gpurun_out/abtree_$f.log
done
grep -H median gpurun_out/abtree_*_train.log
