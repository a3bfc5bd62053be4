#!/bin/bash
# adanalytics (config 5) kernel phases (profiling build) + SQL variants
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out
Q="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100"
PGPU_PROFILE=1 timeout -k 10 200 python3 $R/scripts/kexp.py adanalytics 30 "$Q" \
  "SELECT COUNT(*) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856" > $R/gpurun_out/ad_prof.log 2>&1 || exit 1
grep " ms \|pgpu profile" $R/gpurun_out/ad_prof.log | sort | uniq -c | sort -rn | head -6 | cut -c1-420
