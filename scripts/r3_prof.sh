#!/bin/bash
# Kernel-trace stats of the bench workloads (one rocprofv3 run each), then PMC passes (one counter block per run)
# for the workloads in $PMC_WLS.  Usage: r3_prof.sh <tag>   (WLS / PMC_WLS / PMC_COUNTERS override the lists)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
for wl in ${WLS:-adanalytics range_in bitmap5 groupby1m groupby1m_zipf}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$wl" -o run -- \
    python3 $BENCH --workload $wl --steps ${STEPS:-10} --warmup 2 > "$OUT/$wl.log" 2>&1 || { echo "trace $wl failed rc=$?"; tail -5 "$OUT/$wl.log"; exit 1; }
  grep -h '"metric"' "$OUT/$wl.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_avg'],3), round(d['roofline']['frac'],3))"
done
for wl in ${PMC_WLS:-}; do
  for c in ${PMC_COUNTERS:-FETCH_SIZE WRITE_SIZE SQ_LDS_BANK_CONFLICT}; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${wl}_$c" -o run -- \
      python3 $BENCH --workload $wl --steps 3 --warmup 1 > "$OUT/pmc_${wl}_$c.log" 2>&1 || { echo "pmc $wl $c failed rc=$?"; exit 1; }
  done
done

# phase counters of the profiling build (PGPU_PROFILE=1: libpinotgpu_prof.so) for $PROF_WLS
for wl in ${PROF_WLS:-}; do
  PGPU_PROFILE=1 timeout -k 10 200 python3 $BENCH --workload $wl --steps 3 --warmup 1 > "$OUT/phase_$wl.log" 2>&1 \
    || { echo "phase $wl failed rc=$?"; tail -5 "$OUT/phase_$wl.log"; exit 1; }
  grep "pgpu profile" "$OUT/phase_$wl.log" | tail -2
done
echo done
