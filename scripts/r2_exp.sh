#!/bin/bash
# Round-2 experiments on the GPU box: cancel tests, config-5 kernel time with / without nt tile DMAs, phase profile.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2exp
Q5="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100"
QC="SELECT COUNT(*) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856"
timeout -k 10 300 python -u -m pytest tests/test_gpu_cancel.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r2exp/cancel.log 2>&1
echo "cancel rc=$?"; tail -3 gpurun_out/r2exp/cancel.log
timeout -k 10 200 python3 scripts/kexp.py adanalytics 30 "$Q5" "$QC" > gpurun_out/r2exp/k_default.log 2>&1 || exit 1
PGPU_DIRECT_NT=1 timeout -k 10 200 python3 scripts/kexp.py adanalytics 30 "$Q5" "$QC" > gpurun_out/r2exp/k_nt.log 2>&1 || exit 1
cat gpurun_out/r2exp/k_default.log gpurun_out/r2exp/k_nt.log | grep " ms "
PGPU_PROFILE=1 timeout -k 10 200 python3 scripts/kexp.py adanalytics 30 "$Q5" "$QC" > gpurun_out/r2exp/k_prof.log 2>&1 || exit 1
grep " ms \|pgpu profile" gpurun_out/r2exp/k_prof.log | sort | uniq -c | sort -rn | head -6 | cut -c1-400
