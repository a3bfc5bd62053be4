#!/bin/bash
# Ring-kernel phase counters (profiling build) for config 2 and config 3 and their SUM-free variants.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out/r2exp6
F2="r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)"
F3="(a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)"
PGPU_PROFILE=1 timeout -k 10 200 python3 $R/scripts/kexp.py range_in 30 "SELECT COUNT(*), SUM(m) FROM synth WHERE $F2" \
  "SELECT SUM(m) FROM synth" > $R/gpurun_out/r2exp6/c2.log 2>&1 || exit 1
PGPU_PROFILE=1 timeout -k 10 200 python3 $R/scripts/kexp.py bitmap5 30 "SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE $F3" \
  "SELECT COUNT(*) FROM bitmap5 WHERE $F3" > $R/gpurun_out/r2exp6/c3.log 2>&1 || exit 1
for f in c2 c3; do grep " ms \|pgpu profile" $R/gpurun_out/r2exp6/$f.log | sort | uniq -c | sort -rn | head -6 | cut -c1-500; done
