#!/bin/bash
# HBM-traffic profile of bench workloads: kernel-trace stats, FETCH_SIZE and WRITE_SIZE passes (one TCC
# counter per pass), the FETCH_SIZE calibration pass on config 5's filter stream when adanalytics is listed, and
# with LDS=1 an SQ pass of LDS counters.  Summaries: python scripts/pmc_summarize.py <tag>_<wl> <wl>.
# Usage: pmc.sh <tag> "<workloads>"
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; WLS=$2
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
for WL in $WLS; do
  OUT=$R/gpurun_out/${TAG}_$WL; mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 $BENCH --workload $WL --steps ${STEPS:-10} --warmup 2 --full-out "$OUT/trace.json" > "$OUT/trace.log" 2>&1 || { echo "trace $WL failed rc=$?"; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run -- \
      python3 $BENCH --workload $WL --steps 3 --warmup 1 --full-out "$OUT/pmc_$c.json" > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $WL $c failed rc=$?"; exit 1; }
  done
  if [ "$WL" = adanalytics ]; then
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_cal" -o run -- \
      python3 $BENCH --workload adanalytics_count --steps 3 --warmup 1 --full-out "$OUT/pmc_cal.json" > "$OUT/pmc_cal.log" 2>&1 || { echo "pmc cal failed rc=$?"; exit 1; }
  fi
  if [ "${LDS:-0}" = 1 ]; then
    timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv \
      -d "$OUT/pmc_lds" -o run -- python3 $BENCH --workload $WL --steps 3 --warmup 1 --full-out "$OUT/pmc_lds.json" > "$OUT/pmc_lds.log" 2>&1 || { echo "pmc lds $WL failed rc=$?"; exit 1; }
  fi
  echo "$WL profiled"
done
echo done
