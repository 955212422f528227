# Same-box A/B of the library before the XCD-local work (ab/prexl.so, built from commit 4d71023's
# sources) against the in-tree build with XCD-local groups off / on, alternating processes:
# per-kernel times of the C2 / C5 forwards (scripts/persist_hook_ab.py) and the C5 bench batch
set -e
mkdir -p gpurun_out
for i in 1 2; do
  AUTOVC_HIP_LIB=ab/prexl.so timeout -k 10 150 python scripts/persist_hook_ab.py avc_lstm_persist_depth 2 2 >> gpurun_out/abpre_old.log 2>&1
  timeout -k 10 150 python scripts/persist_hook_ab.py avc_lstm_persist_xcd 0 1 >> gpurun_out/abpre_new.log 2>&1
  AUTOVC_HIP_LIB=ab/prexl.so timeout -k 10 150 python scripts/long_hook_ab.py avc_lstm_persist_depth 2 >> gpurun_out/abpre_old_long.log 2>&1
  timeout -k 10 150 python scripts/long_hook_ab.py avc_lstm_persist_xcd 0 1 >> gpurun_out/abpre_new_long.log 2>&1
done
grep -H "per forward" gpurun_out/abpre_*.log
