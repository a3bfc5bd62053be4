#!/bin/bash
# rocprofv3 kernel-trace stats of bench workloads at the current build (no tests).  Usage: profile.sh <tag> "<workloads>"
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; WLS=$2
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
for wl in $WLS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$wl" -o run -- \
    python3 $BENCH --workload $wl --steps ${STEPS:-10} --warmup 2 > "$OUT/$wl.log" 2>&1 || { echo "trace $wl failed rc=$?"; tail -5 "$OUT/$wl.log"; exit 1; }
  grep -h '"metric"' "$OUT/$wl.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_avg'],3), round(d['roofline']['frac'],3))"
done
echo done
