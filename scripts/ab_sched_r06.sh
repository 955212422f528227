export REF_WGRAD=1
timeout -k 10 600 bash scripts/compare_libs.sh ab/r06c.so > gpurun_out/cmp6c.log 2>&1 || exit $?
tail -6 gpurun_out/cmp6c.log
for l in ab/r06c.so abd_gilp/libautovc_hip.so abd_gmc/libautovc_hip.so; do
  echo "== $l"
  timeout -k 10 300 bash scripts/ab_r05.sh $l > gpurun_out/absc.log 2>&1 || exit $?
  tail -4 gpurun_out/absc.log
  timeout -k 10 300 bash scripts/ab_lib_train.sh $l 2>&1 | grep median
done
for l in abd_lilp/libautovc_hip.so abd_eilp/libautovc_hip.so; do
  echo "== $l"
  timeout -k 10 300 bash scripts/ab_r05.sh $l > gpurun_out/absc.log 2>&1 || exit $?
  tail -4 gpurun_out/absc.log
  timeout -k 10 300 bash scripts/ab_lib_train.sh $l 2>&1 | grep median
done
