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
