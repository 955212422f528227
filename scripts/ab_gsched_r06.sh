# gemm.hip on the max-ILP / max-memory-clause schedulers (abd_gilp / abd_gmc) against the in-tree build
export REF_WGRAD=1
for d in abd_gilp abd_gmc; do
  echo "== $d"
  timeout -k 10 300 bash scripts/ab_r05.sh $d/libautovc_hip.so > gpurun_out/abgs.log 2>&1 || exit $?
  tail -4 gpurun_out/abgs.log
  timeout -k 10 300 bash scripts/ab_lib_train.sh $d/libautovc_hip.so 2>&1 | grep median
done
