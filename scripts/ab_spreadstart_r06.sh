# the spread LDS-DMA pieces issued from chunk 1 (abd_st1) or chunk 2 (abd_st2) instead of chunk 0
export REF_WGRAD=1
for d in abd_st1 abd_st2; do
  echo "== $d"
  timeout -k 10 300 bash scripts/ab_r05.sh $d/libautovc_hip.so > gpurun_out/abst.log 2>&1 || exit $?
  tail -4 gpurun_out/abst.log
  timeout -k 10 300 bash scripts/ab_lib_train.sh $d/libautovc_hip.so 2>&1 | grep median
done
