export REF_WGRAD=1
timeout -k 10 600 bash scripts/compare_libs.sh ab/r06d.so > gpurun_out/cmp6d.log 2>&1 || exit $?
tail -6 gpurun_out/cmp6d.log
timeout -k 10 300 bash scripts/ab_r05.sh ab/r06d.so > gpurun_out/absd.log 2>&1 || exit $?
tail -4 gpurun_out/absd.log
timeout -k 10 300 bash scripts/ab_lib_train.sh ab/r06d.so 2>&1 | grep median
