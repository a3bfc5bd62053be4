#!/bin/bash
# Kernel-trace statistics of the secondary workloads (configs 2, 3, 4): per-kernel durations for the phase split.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for WL in ${WLS:-groupby1m range_in bitmap5}; do
  OUT=$R/gpurun_out/r2wl/$WL; mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-check --no-secondary --workload $WL --steps 10 --warmup 2 \
    > "$OUT/trace.log" 2>&1 || { echo "trace $WL failed rc=$?"; exit 1; }
  echo "== $WL"; head -8 "$OUT/run_kernel_stats.csv" | cut -c1-160
done
