#!/bin/bash
# Inverted-leaf expansion (invexp_kernel): config 3 and config 5-inv kernel times with and without, then GPU tests.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2exp7
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > gpurun_out/r2exp7/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep " ms \|passed\|failed" gpurun_out/r2exp7/$name.log | tail -6 | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
F3="(a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)"
Q5="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100"
step c3 300 python3 scripts/kexp.py bitmap5 30 "SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE $F3" \
  "SELECT COUNT(*) FROM bitmap5 WHERE $F3" "SELECT COUNT(*) FROM bitmap5 WHERE a = 10 AND b IN (30, 70)"
PGPU_NO_INVEXP=1 step c3_off 300 python3 scripts/kexp.py bitmap5 30 "SELECT COUNT(*) FROM bitmap5 WHERE $F3"
  "SELECT COUNT(*) FROM bitmap5 WHERE $F3" "SELECT COUNT(*) FROM bitmap5 WHERE a = 10 AND b IN (30, 70)"
step c5inv 300 python3 scripts/kexp.py adanalytics_inv 30 "$Q5"
PGPU_NO_INVEXP=1 step c5inv_off 300 python3 scripts/kexp.py adanalytics_inv 30 "$Q5"
step tests 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
