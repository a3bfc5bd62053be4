#!/bin/bash
# Phase 2 of the partitioned group-by with the frame-of-reference dictionary in LDS (config 4), then the GPU suite.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2exp9
Q4="SELECT k, SUM(m), MAX(m), COUNT(*) FROM synth GROUP BY k ORDER BY SUM(m) DESC LIMIT 100"
timeout -k 10 300 python3 scripts/kexp.py groupby1m 60 "$Q4" > gpurun_out/r2exp9/for.log 2>&1 || { echo "for rc=$?"; tail -20 gpurun_out/r2exp9/for.log; exit 1; }
PGPU_NO_FOR=1 timeout -k 10 300 python3 scripts/kexp.py groupby1m 60 "$Q4" > gpurun_out/r2exp9/nofor.log 2>&1 || exit 1
grep -h " ms " gpurun_out/r2exp9/for.log gpurun_out/r2exp9/nofor.log | cut -c1-120
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r2exp9/tests.log 2>&1 \
  || { echo "tests failed rc=$?"; tail -30 gpurun_out/r2exp9/tests.log; exit 1; }
tail -1 gpurun_out/r2exp9/tests.log
