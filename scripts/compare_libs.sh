# Bit-identity of the in-tree build against a saved library (argv[1]): conversion forwards and
# gradients (compare_fwd.py) and two C3 training steps (compare_train.py).
set -e
lib=$1
mkdir -p gpurun_out
AUTOVC_WGRAD_IMAGE=${REF_WGRAD:-0} AUTOVC_HIP_LIB=$lib timeout -k 10 200 python scripts/compare_fwd.py gpurun_out/cmpf_ref.pt
timeout -k 10 200 python scripts/compare_fwd.py gpurun_out/cmpf_new.pt
AUTOVC_WGRAD_IMAGE=${REF_WGRAD:-0} AUTOVC_HIP_LIB=$lib timeout -k 10 200 python scripts/compare_train.py gpurun_out/cmpt_ref.pt
timeout -k 10 200 python scripts/compare_train.py gpurun_out/cmpt_new.pt
python scripts/compare_train.py --diff gpurun_out/cmpf_ref.pt gpurun_out/cmpf_new.pt | grep -c bit-identical || true
python scripts/compare_train.py --diff gpurun_out/cmpf_ref.pt gpurun_out/cmpf_new.pt | grep DIFFERENT || true
python scripts/compare_train.py --diff gpurun_out/cmpt_ref.pt gpurun_out/cmpt_new.pt
rm -f gpurun_out/cmpf_*.pt gpurun_out/cmpt_*.pt
