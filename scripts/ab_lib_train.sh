# Same-box A/B of a saved library (argv[1]) against the in-tree build on the C3 training step,
# alternating processes (scripts/train_time.py), three rounds
set -e
for i in 1 2 3; do
  AUTOVC_WGRAD_IMAGE=${REF_WGRAD:-0} AUTOVC_HIP_LIB=$1 timeout -k 10 150 python scripts/train_time.py
  timeout -k 10 150 python scripts/train_time.py
done
