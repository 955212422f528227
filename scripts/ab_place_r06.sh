# placement of the spread LDS-DMA pieces: after the chunk's MFMAs (abd_pl1), interleaved with them
# by sched_group_barrier (abd_pl2), against the in-tree build (before the MFMAs)
export REF_WGRAD=1
for d in abd_pl1 abd_pl2; do
  echo "== $d"
  timeout -k 10 300 bash scripts/ab_r05.sh $d/libautovc_hip.so > gpurun_out/abpl.log 2>&1 || exit $?
  tail -4 gpurun_out/abpl.log
  timeout -k 10 300 bash scripts/ab_lib_train.sh $d/libautovc_hip.so 2>&1 | grep median
done
