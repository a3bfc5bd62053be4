#!/bin/bash
# Instruction-mix profile of bench workloads: one SQ counter pass (VALU / SALU / LDS instructions, LDS and
# any-wait cycles, wave cycles) per workload.  Usage: sqprof.sh <tag> "<workloads>"
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; WLS=$2
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
for WL in $WLS; do
  OUT=$R/gpurun_out/${TAG}_$WL; mkdir -p "$OUT"
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT \
    --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $BENCH --workload $WL --steps 3 --warmup 1 > "$OUT/pmc_sq.log" 2>&1 \
    || { echo "pmc sq $WL failed rc=$?"; exit 1; }
  echo "$WL profiled"
done
echo done
