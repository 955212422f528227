# The BPTT split into its own translation unit (lstm_bptt.hip, default scheduler) with the forward
# recurrences on the max-ILP scheduler: GPU suite, bit-identity and same-box A/B against ab/r06c.so
export REF_WGRAD=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_suite.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/compare_libs.sh ab/r06c.so > gpurun_out/cmp6c.log 2>&1 || exit $?
tail -6 gpurun_out/cmp6c.log
timeout -k 10 300 bash scripts/ab_r05.sh ab/r06c.so > gpurun_out/absc.log 2>&1 || exit $?
tail -4 gpurun_out/absc.log
timeout -k 10 300 bash scripts/ab_lib_train.sh ab/r06c.so 2>&1 | grep median
