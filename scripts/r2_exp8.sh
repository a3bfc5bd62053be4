#!/bin/bash
# Dense (ring kernel, staged SUM column) vs sparse (candidate gathers, self-loading kernel) aggregation on config 2.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2exp8
F2="r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)"
for T in 0.5 1.01; do
  PGPU_DENSE_TOUCH=$T timeout -k 10 300 python3 scripts/kexp.py range_in 30 "SELECT COUNT(*), SUM(m) FROM synth WHERE $F2" \
    "SELECT SUM(m) FROM synth WHERE r BETWEEN 114691 AND 344060" "SELECT SUM(m) FROM synth WHERE i IN (100)" \
    > gpurun_out/r2exp8/t$T.log 2>&1 || exit 1
  echo "== touch $T"; grep " ms " gpurun_out/r2exp8/t$T.log | cut -c1-160
done
PGPU_DENSE_TOUCH=1.01 timeout -k 10 300 python3 scripts/kexp.py bitmap5 30 \
  "SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE (a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)" \
  > gpurun_out/r2exp8/c3.log 2>&1 || exit 1
echo "== c3 touch 1.01"; grep " ms " gpurun_out/r2exp8/c3.log | cut -c1-160
