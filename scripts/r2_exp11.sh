#!/bin/bash
# Config 4 (uniform and Zipf) with the compact frame-of-reference phase 2 at the original geometry, then the suite.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2exp11
Q4="SELECT k, SUM(m), MAX(m), COUNT(*) FROM synth GROUP BY k ORDER BY SUM(m) DESC LIMIT 100"
for W in groupby1m groupby1m_zipf; do
  for F in 0 1; do
    PGPU_NO_FOR=$F timeout -k 10 300 python3 scripts/kexp.py $W 60 "$Q4" > gpurun_out/r2exp11/$W.$F.log 2>&1 \
      || { echo "$W $F rc=$?"; tail -20 gpurun_out/r2exp11/$W.$F.log; exit 1; }
    echo "$W NO_FOR=$F $(grep ' ms ' gpurun_out/r2exp11/$W.$F.log | cut -c1-40)"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r2exp11/tests.log 2>&1 \
  || { echo "tests failed rc=$?"; tail -30 gpurun_out/r2exp11/tests.log; exit 1; }
tail -1 gpurun_out/r2exp11/tests.log
