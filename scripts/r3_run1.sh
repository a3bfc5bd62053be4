#!/bin/bash
# Round-3 GPU pass: the GPU suite + config-4 bench check, kernel traces of every bench workload, the
# profiling build's phase counters for config 4, and the gather-policy micro-benchmark.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
bash scripts/r3_check.sh || exit 1
WLS="${WLS:-adanalytics range_in bitmap5 groupby1m groupby1m_zipf}" PROF_WLS="${PROF_WLS:-groupby1m}" bash scripts/r3_prof.sh ${TAG:-r3a} || exit 1
if [ -x tools/gather_policy_bench ]; then
  timeout -k 10 120 tools/gather_policy_bench > gpurun_out/gather_policy.txt 2>&1 || { echo "gather bench rc=$?"; exit 1; }
  cat gpurun_out/gather_policy.txt
fi
