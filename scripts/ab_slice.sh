#!/bin/bash
# A/B of the bit-sliced filter leaves: phase profile with and without (PGPU_NO_SLICE=1); gpurun_out/ab_slice*.log
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out
T=adAnalytics
Q1="SELECT COUNT(*) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856"
Q2="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch"
PGPU_PROFILE=1 timeout -k 10 200 python3 -u $R/scripts/kexp.py adanalytics 30 "$Q1" "$Q2" > $R/gpurun_out/ab_slice.log 2>&1 || exit 1
PGPU_NO_SLICE=1 PGPU_PROFILE=1 timeout -k 10 200 python3 -u $R/scripts/kexp.py adanalytics 30 "$Q1" "$Q2" > $R/gpurun_out/ab_noslice.log 2>&1 || exit 1
grep -h " ms " $R/gpurun_out/ab_slice.log $R/gpurun_out/ab_noslice.log
