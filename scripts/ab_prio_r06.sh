# gemm16f with the younger half of its waves at s_setprio 1 in the K loop (abd_prio) against in-tree
export REF_WGRAD=1
timeout -k 10 300 bash scripts/ab_r05.sh abd_prio/libautovc_hip.so > gpurun_out/abpr.log 2>&1 || exit $?
tail -4 gpurun_out/abpr.log
timeout -k 10 300 bash scripts/ab_lib_train.sh abd_prio/libautovc_hip.so 2>&1 | grep median
