#!/bin/bash
# A/B of bench workloads under env knobs with rocprofv3 kernel stats: per knob set, the average ms of every kernel
# whose name matches $KPAT (default: the partitioned group-by phases).
# Usage: abprof.sh <tag> "<workloads>" "<knob-set-1>" "<knob-set-2>" ...   (a knob set: "A=1 B=2" or "-")
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; WLS=$2; shift 2
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
cd /tmp && export TMPDIR=/tmp
for wl in $WLS; do
  i=0
  for knobs in "$@"; do
    i=$((i+1))
    for kv in $knobs; do [ "$kv" != "-" ] && export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${wl}_$i" -o run -- \
      python3 $BENCH --workload $wl --steps ${STEPS:-5} --warmup 2 > "$OUT/${wl}_$i.log" 2>&1 \
      || { echo "$wl [$knobs] failed rc=$?"; tail -5 "$OUT/${wl}_$i.log"; exit 1; }
    for kv in $knobs; do [ "$kv" != "-" ] && unset "${kv%%=*}"; done
    python3 - "$OUT/${wl}_$i/run_kernel_stats.csv" "$wl [$knobs]" "${KPAT:-part_}" <<'EOF'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = [f"{r['Name'].split('(')[0].split('::')[-1][:48]} {float(r['AverageNs']) / 1e6:.3f}"
       for r in rows if re.search(sys.argv[3], r['Name'])]
print(sys.argv[2], " | ".join(out))
EOF
  done
done
echo done
