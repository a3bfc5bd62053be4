#!/bin/bash
# Config 4 A/B: groupby1m and groupby1m_zipf with and without phase 2's hot-key registers (PGPU_NO_HOTKEYS=1),
# rocprof kernel stats of each.  Usage: ab_groupby.sh <tag>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for wl in ${WLS:-groupby1m_zipf groupby1m}; do
  for hot in 1 0; do
    name=${wl}_hot$hot
    if [ $hot = 0 ]; then export PGPU_NO_HOTKEYS=1; else unset PGPU_NO_HOTKEYS; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
      python3 $R/bench.py --no-cpu-baseline --no-check --no-secondary --workload $wl --steps ${STEPS:-10} --warmup 2 \
      --full-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1 || { echo "trace $name failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
    grep -h '"metric"' "$OUT/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_avg'],3), round(d['roofline']['frac'],3))"
  done
done
unset PGPU_NO_HOTKEYS
echo done
