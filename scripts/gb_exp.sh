#!/bin/bash
# Group-by 1M experiments on the GPU box: SQL variants, phase profile (profiling build), SQ counter passes.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/gbexp; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
Q1="SELECT k, SUM(m), MAX(m), COUNT(*) FROM synth GROUP BY k ORDER BY SUM(m) DESC LIMIT 100"
timeout -k 10 200 python3 $R/scripts/kexp.py groupby1m 30 "$Q1" "SELECT k, COUNT(*) FROM synth GROUP BY k" \
  "SELECT k, SUM(m) FROM synth GROUP BY k" "SELECT COUNT(*), SUM(m), MAX(m) FROM synth" > $OUT/variants.log 2>&1 || exit 1
PGPU_PROFILE=1 timeout -k 10 200 python3 $R/scripts/kexp.py groupby1m 30 "$Q1" > $OUT/prof.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_ATOMIC_RETURN" \
           "WRITE_SIZE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p$i -- python3 $R/scripts/kexp.py groupby1m 30 "$Q1" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
