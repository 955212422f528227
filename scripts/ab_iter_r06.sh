# lstm_persist.hip on the iterative-ILP scheduler (abd_it) against the in-tree max-ILP build
timeout -k 10 300 bash scripts/ab_r05.sh abd_it/libautovc_hip.so > gpurun_out/abit.log 2>&1 || exit $?
tail -4 gpurun_out/abit.log
