# gemm16f's next-tile LDS-DMA spread over 2 / 4 chunks (abd_sp2 / abd_sp4) against the in-tree build
export REF_WGRAD=1
for d in abd_sp2 abd_sp4; do
  echo "== $d"
  timeout -k 10 300 bash scripts/ab_r05.sh $d/libautovc_hip.so > gpurun_out/absp.log 2>&1 || exit $?
  tail -4 gpurun_out/absp.log
  timeout -k 10 300 bash scripts/ab_lib_train.sh $d/libautovc_hip.so 2>&1 | grep median
done
