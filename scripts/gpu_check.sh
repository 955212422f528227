#!/bin/bash
# GPU-box check sequence: every step has its own time limit; a test failure (exit 1) lets the
# sequence continue, anything else (fault, abort, segfault, timeout) ends it immediately.
set -u
export PYTHONUNBUFFERED=1
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    persist) run persist 300 python -u -m pytest tests/test_gpu_model.py -x -v -s -k persistent --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    bnf)   run bnf 300 python -u -m pytest tests/test_gpu_bnfuse.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    safety) run safety 300 python -u -m pytest tests/test_gpu_persist_safety.py tests/test_gpu_coresidency.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    kern)  run kern 600 python -m pytest tests/test_gpu_kernels.py -v -m gpu -x --timeout 120 -p no:cacheprovider ;;
    model) run model 600 python -m pytest tests/test_gpu_model.py -v -m gpu -s --timeout 200 -p no:cacheprovider ;;
    gpu)   run gpu 900 python -m pytest tests -v -m gpu --timeout 300 -p no:cacheprovider ;;
    bench) run bench 400 python bench.py --steps 10 --warmup 2 ;;
    benchdef) run benchdef 400 python bench.py ;;
    benchnt) run benchnt 400 python bench.py --steps 20 --warmup 3 --no-timing --no-cpu ;;
    perf)  run perf 400 python scripts/perf_layers.py 1 6 7 ;;
    prof)  run prof 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o fwd -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-timing ;;
    pmcf)  run pmcf 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF -o fwd -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-timing ;;
    pmcw)  run pmcw 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW -o fwd -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-timing ;;
    pmcft) run pmcft 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcFT -o train -- python3 bench.py --mode train --steps 2 --warmup 1 --no-cpu --no-timing ;;
    pmcwt) run pmcwt 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcWT -o train -- python3 bench.py --mode train --steps 2 --warmup 1 --no-cpu --no-timing ;;
    ktrain) run ktrain 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktrain -o train -- python3 bench.py --mode train --steps 1 --warmup 1 --no-cpu --no-timing ;;
    proftrain) run proftrain 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/proftrain -o train -- python3 bench.py --mode train --steps 3 --warmup 1 --no-cpu --no-timing ;;
    sstamps) run sstamps 300 python scripts/stamps_split.py 0:0 0:4 ;;
    pstamps) run pstamps 300 python scripts/stamps_persist.py 1 ;;
    pstamps2) run pstamps2 300 python scripts/stamps_persist.py 2 ;;
    pstampsd1) run pstampsd1 300 python scripts/stamps_persist.py 1 1 ;;
    pstampsd2) run pstampsd2 300 python scripts/stamps_persist.py 1 2 ;;
    pstampsd4) run pstamps 300 python scripts/stamps_persist.py 2 && run pstampsd4 300 python scripts/stamps_persist.py 2 4 ;;
    gcfg) run gcfg 300 python scripts/gemm_cfgs.py ;;
    pmodes) run pmodes 300 python scripts/persist_modes.py ;;
    pmodes1) run pmodes1 300 python scripts/persist_modes.py 1 0 1 1 ;;
    pident) run pident 300 python scripts/persist_identity.py ;;
    pdepth) run pdepth 300 python scripts/persist_modes.py 0 2:1 2:2 2:1 2:2 1:2 ;;
    probe) run probe 200 python scripts/probe_cache.py ;;
    gpmc)  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
             n=$(echo $grp | cut -d' ' -f1); run gpmc_$n 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/gpmc/$n -o g -- python3 scripts/gemm_micro.py; done ;;
    gpmc3) for mode in c2 c3fwd c3bwd; do
             run gtrace_$mode 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gtrace/$mode -o g -- python3 scripts/gemm_micro.py $mode
             for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
               n=$(echo $grp | cut -d' ' -f1); run gpmc3_${mode}_$n 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/gpmc3/${mode}_$n -o g -- python3 scripts/gemm_micro.py $mode; done; done ;;
    stamps) run stamps 300 python scripts/stamps_lstm.py ;;
    audio) run audio 600 python -m pytest tests/test_gpu_audio.py -v -m gpu -s --timeout 200 -p no:cacheprovider ;;
    benchtrain) run benchtrain 400 python bench.py --mode train --steps 5 --warmup 2 --no-cpu ;;
    benchtraincpu) run benchtraincpu 500 python bench.py --mode train --steps 5 --warmup 2 ;;
    benchlong) run benchlong 400 python bench.py --mode long --steps 5 --warmup 2 ;;
    proflong) run proflong 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/proflong -o long -- python3 bench.py --mode long --steps 5 --warmup 2 --no-cpu --no-timing ;;
    benchmel) run benchmel 400 python bench.py --mode mel --steps 10 --warmup 2 ;;
    benchse) run benchse 400 python bench.py --mode se --steps 10 --warmup 2 ;;
    benchvoc) run benchvoc 400 python bench.py --mode vocoder --steps 3 --warmup 1 ;;
    profvoc) run profvoc 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/profvoc -o voc -- python3 bench.py --mode vocoder --steps 2 --warmup 1 --no-cpu --no-timing ;;
    profmel) run profmel 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/profmel -o mel -- python3 bench.py --mode mel --steps 10 --warmup 2 --no-cpu --no-timing ;;
    profse) run profse 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/profse -o se -- python3 bench.py --mode se --steps 10 --warmup 2 --no-cpu --no-timing ;;
    bnfab) run bnfab 300 python scripts/persist_hook_ab.py avc_bn_fuse 1 2 1 2 1 2 ;;
    bnftrain) run bnftrain 400 python scripts/train_hook_ab.py avc_bn_fuse 1 2 ;;
    ebudget) run ebudget 400 python scripts/error_budget.py 2 1 128 && run ebudget0 400 python scripts/error_budget.py 0 1 128 && run ebudget64 600 python scripts/error_budget.py 0 64 128 ;;
    rccl) run rccl 400 python -u -m pytest tests/test_gpu_rccl.py -x -v -s --timeout 600 -p no:cacheprovider ;;
    bnbwd) run bnbwd 400 python -u -m pytest tests/test_gpu_bnbwd.py tests/test_gpu_kernels.py -x -v -s --timeout 200 -p no:cacheprovider ;;
    bnbwdab) run bnbwdab 400 python scripts/train_hook_ab.py avc_bn_bwd_frag 0 1 ;;
    prodcurve) run prodcurve 500 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_curve.py -x -v -s --timeout 300 -p no:cacheprovider ;;
    wrp) run wrp 400 python -u -m pytest tests/test_gpu_wavernn_persist.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider && run wrpab 300 python scripts/vocoder_ab.py 3 ;;
    wrstamps) run wrstamps 300 python scripts/vocoder_stamps.py 128 ;;
    bnstat) run bnstat 600 python -u -m pytest tests/test_gpu_bnfuse.py tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_margin.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    voctest) run voctest 400 python -u -m pytest tests/test_gpu_wavernn.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    dgsplit) run dgsplit 300 python -u -m pytest tests/test_gpu_dgsplit.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider && run dgsplitab 400 python scripts/train_hook_ab.py avc_dg_dual_split 0 1 ;;
    pmclong) run pmcfl 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcFL -o long -- python3 bench.py --mode long --steps 2 --warmup 1 --no-cpu --no-timing && run pmcwl 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcWL -o long -- python3 bench.py --mode long --steps 2 --warmup 1 --no-cpu --no-timing ;;
    abc2) run abc2 700 bash scripts/ab_c2.sh ab/prev_bnstats.so ;;
    dpprod) run dpprod 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_production.py -x -v -s --timeout 400 -p no:cacheprovider ;;
    fragchain) rm -f gpurun_out/abe.log && run fragchain 600 bash scripts/ab_env.sh AUTOVC_FRAG_CHAIN 0 1 ;;
    r5a) run r5a 900 python -u -m pytest tests/test_gpu_bnfuse.py tests/test_gpu_bnbwd.py tests/test_gpu_wavernn_persist.py tests/test_gpu_persist_safety.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    deadh) run deadh 300 python -u -m pytest tests/test_gpu_dead_h.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    margin) run margin 900 python -u -m pytest tests/test_gpu_margin.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    abr4) run abr4 700 bash scripts/ab_c2.sh ab/prev_r04.so ;;
    abr4t) run abr4t 700 bash scripts/ab_train.sh ab/prev_r04.so ;;
    bandab) run bandab 400 python scripts/persist_hook_ab.py avc_bn_fuse_band 0 1 0 1 0 1 ;;
    pmcband) for g in 0 1; do run pmcbandF$g 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcbandF$g -o fwd -- python3 scripts/fwd_hooks.py avc_bn_fuse_band=$g 4 && run pmcbandW$g 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcbandW$g -o fwd -- python3 scripts/fwd_hooks.py avc_bn_fuse_band=$g 4; done ;;
    fix5) run fix5 600 python -u -m pytest tests/test_gpu_bnfuse.py tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bnbwd.py tests/test_gpu_production.py tests/test_gpu_curve.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    l32diag) run l32test 200 python -u -m pytest tests/test_gpu_lstm32.py -v -x --timeout 100 --timeout-method thread -p no:cacheprovider && run l32diag 200 python scripts/lstm32_diag.py ;;
    dualw) run dualw 300 python -u -m pytest tests/test_gpu_dgsplit.py -v -x --timeout 100 --timeout-method thread -p no:cacheprovider && run dualwab 400 python scripts/train_hook_ab.py avc_dg_dual_wide 0 1 ;;
    bxl) run bxl 400 python -u -m pytest tests/test_gpu_bptt_xl.py -v -x -s --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    bxlsuite) run bxlsuite 700 python -u -m pytest tests/test_gpu_bptt_coalesce.py tests/test_gpu_persist_safety.py tests/test_gpu_production.py tests/test_gpu_curve.py tests/test_gpu_dp.py tests/test_gpu_model.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    bxstamps) export AVC_STAMPS_LIB=stampslib/libautovc_hip_stamps.so && run bxstamps 200 python scripts/stamps_bptt_xl.py ;;
    bxtime) run bxtime 300 python scripts/bptt_xl_ab.py 0 1 ;;
    abheadt) run abheadt 600 bash scripts/ab_lib_train.sh ab/prev_head.so ;;
    bptts) run bptts 400 python -u -m pytest tests/test_gpu_bptt_coalesce.py tests/test_gpu_bptt_xl.py tests/test_gpu_persist_safety.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    bxlab) run bxlab 500 python scripts/train_hook_ab.py avc_bptt_xcd 0 1 ;;
    abtree) run abtree 1000 bash scripts/ab_r04_tree.sh ;;
    roundsab) run roundsab 500 python scripts/train_hook_ab.py avc_gemm_plan_rounds 0 1 ;;
    adam) run adam 300 python -u -m pytest tests/test_gpu_persist_safety.py tests/test_gpu_kernels.py -k "skip or adam" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    marginsmall) run marginsmall 900 python -u -m pytest tests/test_gpu_margin.py -k small -v -s --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    eb1) run eb1a 400 python scripts/error_budget.py 1 1 128 6 && run eb1b 400 python scripts/error_budget.py 1 2 64 6 ;;
    kprice) export AVC_STAMPS_LIB=diag6/libautovc_hip_stamps.so && run kprice0 200 python scripts/stamps_persist.py 2 0 && run kprice4 200 python scripts/stamps_persist.py 2 4 && run kprice8 200 python scripts/stamps_persist.py 2 8 && run kprice0b 200 python scripts/stamps_persist.py 2 0 ;;
    ab5) run ab5 900 bash scripts/ab_r05.sh ;;
    hostgpu) run hostgpu 200 python scripts/host_vs_gpu.py ;;
    cmp6a) run cmp6a 900 bash scripts/compare_libs.sh ab/r06a.so ;;
    wgimg) run wgimg 300 python -u -m pytest tests/test_gpu_wgrad_image.py tests/test_gpu_bnfuse.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    cmpl2) run cmpl2 900 bash scripts/compare_libs.sh abd_l2/libautovc_hip.so ;;
    abl2) run abl2 900 bash scripts/ab_r05.sh abd_l2/libautovc_hip.so ;;
    bnfl2) AUTOVC_HIP_LIB=$PWD/abd_l2/libautovc_hip.so run bnfl2 300 python -u -m pytest tests/test_gpu_bnfuse.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    cmp6b) run cmp6b 900 bash scripts/compare_libs.sh ab/r06b.so ;;
    ab6bt) run ab6bt 600 bash scripts/ab_lib_train.sh ab/r06b.so ;;
    ab5t) run ab5t 600 bash scripts/ab_lib_train.sh ab/r05.so ;;
    epist) AUTOVC_HIP_LIB=$PWD/abd_stamps/libautovc_hip.so run epist 200 python scripts/stamps_bnf.py ;;
    ab6at) run ab6at 600 bash scripts/ab_lib_train.sh ab/r06a.so ;;
    psafe) run psafe 600 python -u -m pytest tests/test_gpu_persist_safety.py tests/test_gpu_model.py tests/test_gpu_bptt_xl.py tests/test_gpu_bptt_coalesce.py tests/test_gpu_coresidency.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    ab6a) run ab6a 900 bash scripts/ab_r05.sh ab/r06a.so ;;
    ab6b) run ab6b 900 bash scripts/ab_r05.sh ab/r06b.so ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
