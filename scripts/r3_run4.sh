#!/bin/bash
# GPU suite (prefix pre-filter tests first), config 5 bench check, round profile of config 5 (trace + PMC + calibration).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prefix.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/prefix_tests.log 2>&1 \
  || { echo "prefix tests failed"; tail -40 gpurun_out/prefix_tests.log; exit 1; }
tail -1 gpurun_out/prefix_tests.log
WLS="adanalytics" STEPS=200 bash scripts/r3_check.sh || exit 1
bash scripts/profile_round.sh ${TAG:-r3b} adanalytics || exit 1
for wl in ${PROF_WLS:-range_in bitmap5}; do
  PGPU_PROFILE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-check --no-secondary --workload $wl --steps 3 --warmup 1 \
    > gpurun_out/phase_$wl.log 2>&1 || { echo "phase $wl failed rc=$?"; tail -5 gpurun_out/phase_$wl.log; exit 1; }
  echo "$wl"; grep "pgpu profile" gpurun_out/phase_$wl.log | tail -1
done
