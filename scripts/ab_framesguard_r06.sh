# (round 6, last changes: the frames kernel, then codes folded into the decoder input) in-tree against ab/r06f.so:
# range tests, GPU suite, bit-identity, C2 / C5 A/B
export REF_WGRAD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_range.py -q -s --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "x1e5|passed|failed"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_suite.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/compare_libs.sh ab/r06f.so > gpurun_out/cmp6f.log 2>&1 || exit $?
tail -6 gpurun_out/cmp6f.log
timeout -k 10 300 bash scripts/ab_r05.sh ab/r06f.so > gpurun_out/absf.log 2>&1 || exit $?
tail -4 gpurun_out/absf.log
