# spread start at chunk 1 (in-tree; instances with KC < 3 keep the burst) against ab/r06g.so (start
# 0): GEMM / fused-BN tests, bit-identity, same-box A/B
export REF_WGRAD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bnfuse.py tests/test_gpu_wgrad_image.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/st1tests.log 2>&1; rc=$?
tail -2 gpurun_out/st1tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/compare_libs.sh ab/r06g.so > gpurun_out/cmp6g.log 2>&1 || exit $?
tail -6 gpurun_out/cmp6g.log
timeout -k 10 300 bash scripts/ab_r05.sh ab/r06g.so > gpurun_out/abst.log 2>&1 || exit $?
tail -4 gpurun_out/abst.log
for r in 1 2; do timeout -k 10 300 bash scripts/ab_lib_train.sh ab/r06g.so 2>&1 | grep median; done
