# bn_apply_frag with 1024 / 2048 workgroups (abd_g1024 / abd_g2048) instead of 8192 (in-tree):
# the C5 forward (unfused BN) and C3
export REF_WGRAD=1
for d in abd_g1024 abd_g2048; do
  echo "== $d"
  timeout -k 10 300 bash scripts/ab_r05.sh $d/libautovc_hip.so > gpurun_out/abbn.log 2>&1 || exit $?
  tail -4 gpurun_out/abbn.log
  timeout -k 10 300 bash scripts/ab_lib_train.sh $d/libautovc_hip.so 2>&1 | grep median
done
