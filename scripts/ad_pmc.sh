#!/bin/bash
# adanalytics (config 5) SQ instruction / stall counters, one pass per set
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/adpmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
Q="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100"
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p$i -- python3 $R/scripts/kexp.py adanalytics 30 "$Q" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
