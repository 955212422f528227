# scheduler flags on top of the unit strategies: the BPTT unit (abd_b*, C3) and the forward
# recurrences (abd_p*, C2 / C5), each against the in-tree build
export REF_WGRAD=1
for d in abd_pbias0 abd_prelax abd_pnounc; do
  echo "== $d"
  timeout -k 10 300 bash scripts/ab_r05.sh $d/libautovc_hip.so > gpurun_out/abfl.log 2>&1 || exit $?
  tail -4 gpurun_out/abfl.log
done
for d in abd_bbias0 abd_brelax abd_bnounc; do
  echo "== $d"
  timeout -k 10 300 bash scripts/ab_lib_train.sh $d/libautovc_hip.so 2>&1 | grep median
done
