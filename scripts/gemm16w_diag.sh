export PYTHONUNBUFFERED=1
for r in 1 2; do
for d in "" abd_nl abd_nm; do
  if [ -n "$d" ]; then export AUTOVC_HIP_LIB=$PWD/$d/libautovc_hip.so; else unset AUTOVC_HIP_LIB; fi
  echo "== lib ${d:-default}"
  timeout -k 10 120 python -u scripts/gemm_cfg_ab.py 8 12 2>&1 | grep cfg
done
done
