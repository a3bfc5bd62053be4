#!/bin/bash
# A/B timing of bench workloads under env knobs (kernel HIP-event ms and ms/step), plus the phase counters of the
# profiling build.  Usage: ab.sh <tag> "<workloads>" "<knob-set-1>" "<knob-set-2>" ...   (a knob set: "A=1 B=2"
# or "-" for none)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; WLS=$2; shift 2
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
for wl in $WLS; do
  i=0
  for knobs in "$@"; do
    i=$((i+1))
    ENVS="PGPU_PROFILE=${PROF:-0}"; [ "$knobs" != "-" ] && ENVS="$ENVS $knobs"
    env $ENVS timeout -k 10 240 python3 $BENCH --workload $wl --steps ${STEPS:-10} --warmup 2 > "$OUT/${wl}_$i.log" 2>&1 \
      || { echo "$wl [$knobs] failed rc=$?"; tail -5 "$OUT/${wl}_$i.log"; exit 1; }
    grep -h '"metric"' "$OUT/${wl}_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$wl [$knobs]', round(d['ms_per_step'],3), round(r['kernel_ms_avg'],3), round(r['frac'],3))"
    grep "pgpu profile" "$OUT/${wl}_$i.log" | tail -1
  done
done
echo done
