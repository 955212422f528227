# Round-6 final measurements on the GPU box: PMC traffic of the three bench modes (separate
# FETCH_SIZE / WRITE_SIZE passes, converted by pmc_traffic.py into profiles/r06_pmc_traffic*.json,
# which bench.py then reads for its roofline line), the bench lines (C2 default, C3 with its CPU
# baseline, C5), rocprof kernel statistics of the same commands, and smoke().  Every step has its
# own time limit (scripts/gpu_check.sh); anything but a test failure ends the sequence.
set -u
export PYTHONUNBUFFERED=1
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
S="bash scripts/gpu_check.sh"
$S pmcf pmcw pmcft pmcwt pmclong || exit $?
for m in "pmcF pmcW" "pmcFT pmcWT train" "pmcFL pmcWL long"; do
  set -- $m
  out=gpurun_out/r06_pmc_traffic${3:+_$3}.json
  python scripts/pmc_traffic.py gpurun_out/$1 gpurun_out/$2 $out > /dev/null || exit $?
  cp $out profiles/
done
$S benchdef benchtraincpu benchlong prof proftrain proflong smoke
