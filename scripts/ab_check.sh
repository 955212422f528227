# Library A/B: bit-identity of C3 training steps and the C2 forward between ablib/prev.so and
# the in-tree build, then alternating-process C2 / C3 timings (scripts/ab_fwd.sh)
set -e
prev=${1:-ablib/prev.so}
AUTOVC_HIP_LIB=$prev timeout -k 10 120 python scripts/compare_train.py gpurun_out/ctr_prev.pt
timeout -k 10 120 python scripts/compare_train.py gpurun_out/ctr_new.pt
python scripts/compare_train.py --diff gpurun_out/ctr_prev.pt gpurun_out/ctr_new.pt
timeout -k 10 600 bash scripts/ab_fwd.sh "$prev"
