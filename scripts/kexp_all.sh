#!/bin/bash
# Kernel-time breakdown over the bench workloads (GPU box); output in gpurun_out/kexp_*.log
mkdir -p gpurun_out
T=adAnalytics
timeout -k 10 200 python -u scripts/kexp.py adanalytics 30 \
 "SELECT COUNT(*) FROM $T" \
 "SELECT COUNT(*) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856" \
 "SELECT COUNT(*) FROM $T WHERE accountId IN (123456789)" \
 "SELECT COUNT(*) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789)" \
 "SELECT SUM(clicks) FROM $T" \
 "SELECT SUM(clicks) FROM $T WHERE daysSinceEpoch BETWEEN 17500 AND 17600" \
 "SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100" \
 > gpurun_out/kexp_ad.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/kexp.py range_in 30 \
 "SELECT COUNT(*), SUM(m) FROM synth WHERE r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)" \
 "SELECT COUNT(*) FROM synth WHERE r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)" \
 "SELECT SUM(m) FROM synth" \
 > gpurun_out/kexp_range.log 2>&1 || exit $?
if [ "${1:-}" = "gb" ]; then
timeout -k 10 200 python -u scripts/kexp.py groupby1m 30 \
 "SELECT k, SUM(m), MAX(m), COUNT(*) FROM synth GROUP BY k ORDER BY SUM(m) DESC LIMIT 100" \
 > gpurun_out/kexp_gb.log 2>&1 || exit $?
fi
