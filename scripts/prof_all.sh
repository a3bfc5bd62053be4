#!/bin/bash
# rocprofv3 kernel stats of every bench workload at HEAD (one bench.py process per workload, headline only, no CPU
# leg).  Usage: prof_all.sh <tag> ["<workloads>"]; summaries land in gpurun_out/<tag>/<workload>/run_kernel_stats.csv
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
WLS=${2:-"adanalytics range_in groupby1m bitmap5 groupby1m_zipf adanalytics_inv adanalytics_exact"}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for wl in $WLS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$wl" -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-check --no-secondary --workload $wl --steps ${STEPS:-20} --warmup 3 \
    --full-out "$OUT/$wl.json" > "$OUT/$wl.log" 2>&1 || { echo "trace $wl failed rc=$?"; tail -5 "$OUT/$wl.log"; exit 1; }
  grep -h "timed:" "$OUT/$wl.log" | tail -1
done
echo done
