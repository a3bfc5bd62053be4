#!/bin/bash
# A/B of the direct (self-loading) kernel vs the loader/consumer ring kernel on config 5 shapes
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out
T=adAnalytics
Q1="SELECT COUNT(*) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856"
Q2="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100"
timeout -k 10 200 python3 -u $R/scripts/kexp.py adanalytics 30 "$Q1" "$Q2" > $R/gpurun_out/ab_direct.log 2>&1 || exit 1
PGPU_NO_DIRECT=1 timeout -k 10 200 python3 -u $R/scripts/kexp.py adanalytics 30 "$Q1" "$Q2" > $R/gpurun_out/ab_nodirect.log 2>&1 || exit 1
grep -h " ms " $R/gpurun_out/ab_direct.log $R/gpurun_out/ab_nodirect.log
