# gemm16f with the next-tile LDS-DMA spread over two chunks (in-tree) against ab/r06e.so: GEMM and
# fused-BN tests, bit-identity, same-box A/B
export REF_WGRAD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bnfuse.py tests/test_gpu_wgrad_image.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sp2tests.log 2>&1; rc=$?
tail -2 gpurun_out/sp2tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/compare_libs.sh ab/r06e.so > gpurun_out/cmp6e.log 2>&1 || exit $?
tail -6 gpurun_out/cmp6e.log
timeout -k 10 300 bash scripts/ab_r05.sh ab/r06e.so > gpurun_out/abse.log 2>&1 || exit $?
tail -4 gpurun_out/abse.log
timeout -k 10 300 bash scripts/ab_lib_train.sh ab/r06e.so 2>&1 | grep median
