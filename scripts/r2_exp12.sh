#!/bin/bash
# Candidate-queue flush threshold 512 (was 256): config 5, config 5 inverted, config 2 and config 3 kernel times.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2exp12
Q5="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100"
F2="r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)"
F3="(a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)"
timeout -k 10 200 python3 scripts/kexp.py adanalytics 30 "$Q5" > gpurun_out/r2exp12/c5.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/kexp.py range_in 30 "SELECT COUNT(*), SUM(m) FROM synth WHERE $F2" > gpurun_out/r2exp12/c2.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/kexp.py bitmap5 30 "SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE $F3" > gpurun_out/r2exp12/c3.log 2>&1 || exit 1
grep -h " ms " gpurun_out/r2exp12/*.log | cut -c1-120
