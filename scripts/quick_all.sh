#!/bin/bash
# Kernel ms of the three bench workloads (30 segments each) + group-by variants.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out
timeout -k 10 200 python3 $R/scripts/kexp.py adanalytics 30 \
  "SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100" \
  "SELECT COUNT(*) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856" \
  "SELECT SUM(clicks) FROM adAnalytics" > $R/gpurun_out/quick_ad.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/scripts/kexp.py range_in 30 \
  "SELECT COUNT(*), SUM(m) FROM synth WHERE r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)" > $R/gpurun_out/quick_ri.log 2>&1 || exit 1
timeout -k 10 200 python3 $R/scripts/kexp.py groupby1m 30 \
  "SELECT k, SUM(m), MAX(m), COUNT(*) FROM synth GROUP BY k ORDER BY SUM(m) DESC LIMIT 100" \
  "SELECT k, COUNT(*) FROM synth GROUP BY k" "SELECT COUNT(*), SUM(m), MAX(m) FROM synth" > $R/gpurun_out/quick_gb.log 2>&1 || exit 1
cat $R/gpurun_out/quick_*.log | grep " ms "
