#!/bin/bash
# range_in (config 2) breakdown: SQL variants + phase profile of the bench query.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out
Q="SELECT COUNT(*), SUM(m) FROM synth WHERE r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)"
timeout -k 10 200 python3 $R/scripts/kexp.py range_in 30 "$Q" \
  "SELECT COUNT(*) FROM synth WHERE r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)" \
  "SELECT COUNT(*) FROM synth WHERE r BETWEEN 114691 AND 344060" \
  "SELECT COUNT(*) FROM synth WHERE i IN (100, 500, 900)" \
  "SELECT COUNT(*), SUM(m) FROM synth WHERE i IN (100, 500, 900)" \
  "SELECT COUNT(*), SUM(m) FROM synth" > $R/gpurun_out/ri_variants.log 2>&1 || exit 1
PGPU_PROFILE=1 timeout -k 10 200 python3 $R/scripts/kexp.py range_in 30 "$Q" "SELECT COUNT(*) FROM synth WHERE r BETWEEN 114691 AND 344060" > $R/gpurun_out/ri_prof.log 2>&1 || exit 1
grep " ms " $R/gpurun_out/ri_variants.log; grep "pgpu profile" $R/gpurun_out/ri_prof.log | sort -u | head -4
