# GEMM diagnostic builds ("Where the GEMM's time goes").
#   bash scripts/gemm_diag_ab.sh build   # here, on the CPU: abd_*/libautovc_hip.so (git-ignored); GEMM_DIAGS
#                                          # picks the builds, e.g. "NOLOAD+DIAG_NOMFMA:nlnm" (flags joined by +)
#   bash scripts/gemm_diag_ab.sh         # on the GPU box: scripts/gemm_cfg_ab.py against each build
set -e
if [ "$1" = build ]; then
  for v in ${GEMM_DIAGS:-NOLOAD:nl DIAG_NOREAD:nr DIAG_NOBAR:nb DIAG_NOMFMA:nm}; do
    d=abd_${v##*:}; mkdir -p $d
    defs=""; for f in $(echo ${v%%:*} | tr '+' ' '); do defs="$defs -DAVC_GEMM_$f=1"; done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-variable \
      $defs -c autovc_amd/csrc/gemm.hip -o $d/gemm.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls build/*.o | grep -v '/gemm.o$') $d/gemm.o \
      -o $d/libautovc_hip.so
    rm $d/gemm.o
  done
  exit 0
fi
for r in 1 2; do
  for d in "" ${GEMM_DIAG_DIRS:-abd_nl abd_nr abd_nb abd_nm}; do
    if [ -n "$d" ]; then export AUTOVC_HIP_LIB=$PWD/$d/libautovc_hip.so; else unset AUTOVC_HIP_LIB; fi
    echo "== lib ${d:-default}"
    timeout -k 10 120 python -u scripts/gemm_cfg_ab.py 8 8 2>&1 | grep cfg | tail -1
  done
done
