#!/bin/bash
# Per-wave phase counters (libpinotgpu_prof.so, PGPU_PROFILE=1) of bench workloads, each with and without an env
# knob.  Usage: phase.sh <tag> "<workloads>" "<KNOB=value>"
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; WLS=$2; KNOB=${3:-}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
for wl in $WLS; do
  for variant in base knob; do
    if [ $variant = knob ] && [ -z "$KNOB" ]; then continue; fi
    ENVS="PGPU_PROFILE=1"; [ $variant = knob ] && ENVS="$ENVS $KNOB"
    env $ENVS timeout -k 10 200 python3 $BENCH --workload $wl --steps 3 --warmup 1 > "$OUT/phase_${wl}_$variant.log" 2>&1 \
      || { echo "phase $wl $variant failed rc=$?"; tail -5 "$OUT/phase_${wl}_$variant.log"; exit 1; }
    echo "$wl $variant:"; grep "pgpu profile" "$OUT/phase_${wl}_$variant.log" | tail -1
  done
done
echo done
