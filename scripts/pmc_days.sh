#!/bin/bash
# SQ counter passes over one filter query (GPU box); output under gpurun_out/pmc_days/
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc_days; cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
Q="SELECT COUNT(*) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856"
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc_days/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_days/p$i -o p$i -- python3 $R/scripts/kexp.py adanalytics 30 "$Q" > $R/gpurun_out/pmc_days/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_days/p$i.log; }
done
