#!/bin/bash
# GPU suite, bench checks of $WLS, phase counters of config 4, gather-policy micro-benchmark.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
WLS="${WLS:-adanalytics groupby1m groupby1m_zipf}" STEPS=${STEPS:-50} bash scripts/r3_check.sh || exit 1
for wl in ${PROF_WLS:-groupby1m}; do
  PGPU_PROFILE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-check --no-secondary --workload $wl --steps 3 --warmup 1 \
    > gpurun_out/phase_$wl.log 2>&1 || { echo "phase $wl failed rc=$?"; tail -5 gpurun_out/phase_$wl.log; exit 1; }
  grep "pgpu profile" gpurun_out/phase_$wl.log | tail -1
done
if [ -x tools/gather_policy_bench ]; then
  timeout -k 10 120 tools/gather_policy_bench > gpurun_out/gather_policy.txt 2>&1 || { echo "gather bench rc=$?"; exit 1; }
  cat gpurun_out/gather_policy.txt
fi
