#!/bin/bash
# GPU suite, then the configs 2 / 3 / 5 kernel times of the current build.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2check
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r2check/tests.log 2>&1 \
  || { echo "tests failed rc=$?"; tail -30 gpurun_out/r2check/tests.log; exit 1; }
tail -2 gpurun_out/r2check/tests.log
F2="r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)"
F3="(a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)"
timeout -k 10 200 python3 scripts/kexp.py range_in 30 "SELECT COUNT(*), SUM(m) FROM synth WHERE $F2" "SELECT SUM(m) FROM synth" \
  > gpurun_out/r2check/c2.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/kexp.py bitmap5 30 "SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE $F3" \
  > gpurun_out/r2check/c3.log 2>&1 || exit 1
grep -h " ms " gpurun_out/r2check/c2.log gpurun_out/r2check/c3.log | cut -c1-160
