#!/bin/bash
# GPU suite + bench checks of $WLS + the gather-policy micro-benchmark.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
WLS="${WLS:-adanalytics groupby1m}" STEPS=${STEPS:-50} bash scripts/r3_check.sh || exit 1
if [ -x tools/gather_policy_bench ]; then
  timeout -k 10 120 tools/gather_policy_bench > gpurun_out/gather_policy.txt 2>&1 || { echo "gather bench rc=$?"; exit 1; }
  cat gpurun_out/gather_policy.txt
fi
