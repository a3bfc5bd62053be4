#!/bin/bash
# Round profile of the bench command on the GPU box: kernel-trace stats, then one PMC pass per TCC counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass).  Usage: profile_round.sh <tag> [workload]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; WL=${2:-adanalytics}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --workload $WL --no-cpu-baseline --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 $BENCH --steps 20 --warmup 3 > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- \
    python3 $BENCH --steps 3 --warmup 1 > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed rc=$?"; exit 1; }
done
echo done
