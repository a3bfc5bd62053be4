#!/bin/bash
# Direct-kernel geometry sweep (slots per wave x workgroups per CU) on config 5 shapes; gpurun_out/sweep_direct.log
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out
T=adAnalytics
Q1="SELECT COUNT(*) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856"
Q2="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100"
: > $R/gpurun_out/sweep_direct.log
for cfg in ${SWEEP:-"2 2" "5 2" "3 4" "2 4"}; do
  set -- ${cfg/_/ }
  echo "== slots $1 wgs $2" >> $R/gpurun_out/sweep_direct.log
  PGPU_DIRECT_SLOTS=$1 PGPU_DIRECT_WGS=$2 timeout -k 10 120 python3 -u $R/scripts/kexp.py adanalytics 30 "$Q1" "$Q2" 2>&1 | grep " ms " >> $R/gpurun_out/sweep_direct.log || exit 1
done
echo "== ring" >> $R/gpurun_out/sweep_direct.log
PGPU_NO_DIRECT=1 timeout -k 10 120 python3 -u $R/scripts/kexp.py adanalytics 30 "$Q1" "$Q2" 2>&1 | grep " ms " >> $R/gpurun_out/sweep_direct.log
if [ -n "$PROF" ]; then
  PGPU_PROFILE=1 PGPU_DIRECT_SLOTS=3 PGPU_DIRECT_WGS=4 timeout -k 10 120 python3 -u $R/scripts/kexp.py adanalytics 30 "$Q1" "$Q2" > $R/gpurun_out/prof_direct.log 2>&1
fi
cat $R/gpurun_out/sweep_direct.log
