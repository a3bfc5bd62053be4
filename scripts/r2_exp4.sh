#!/bin/bash
# Register-direct kernel templated on its plane count: config 5 / COUNT kernel times per workgroups-per-CU.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2exp4
Q5="SELECT daysSinceEpoch, SUM(clicks), SUM(impressions) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856 AND accountId IN (123456789) GROUP BY daysSinceEpoch ORDER BY SUM(impressions) DESC LIMIT 100"
QC="SELECT COUNT(*) FROM adAnalytics WHERE daysSinceEpoch BETWEEN 17849 AND 17856"
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > gpurun_out/r2exp4/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep " ms \|passed\|failed" gpurun_out/r2exp4/$name.log | tail -4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step k_rdirect 200 python3 scripts/kexp.py adanalytics 30 "$Q5" "$QC"
PGPU_DIRECT_WGS=2 step k_wg2 200 python3 scripts/kexp.py adanalytics 30 "$Q5" "$QC"
PGPU_DIRECT_WGS=3 step k_wg3 200 python3 scripts/kexp.py adanalytics 30 "$Q5" "$QC"
step mvtests 300 python -u -m pytest tests/test_mv_columns.py -m gpu -q -x --timeout 120 --timeout-method thread
step tests 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
