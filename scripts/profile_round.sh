#!/bin/bash
# Round profile of the bench command on the GPU box: kernel-trace stats, then one PMC pass per TCC counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass), plus a FETCH_SIZE pass over config 5's filter stream alone
# (adanalytics_count: a known byte count, the calibration of FETCH_SIZE for this access width -- MI355X_MICROARCH.md
# "Other access widths are uncalibrated").  Usage: profile_round.sh <tag> [workload]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; WL=${2:-adanalytics}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 $BENCH --workload $WL --steps 20 --warmup 3 > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- \
    python3 $BENCH --workload $WL --steps 3 --warmup 1 > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed rc=$?"; exit 1; }
done
if [ "$WL" = adanalytics ]; then
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_cal" -o run -- \
    python3 $BENCH --workload adanalytics_count --steps 3 --warmup 1 > "$OUT/pmc_cal.log" 2>&1 || { echo "pmc cal failed rc=$?"; exit 1; }
fi
echo done
