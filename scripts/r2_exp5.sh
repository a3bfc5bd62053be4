#!/bin/bash
# Config 2 / config 3 kernel-time decomposition by query variant.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
mkdir -p gpurun_out/r2exp5
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > gpurun_out/r2exp5/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep " ms " gpurun_out/r2exp5/$name.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
F2="r BETWEEN 114691 AND 344060 AND i IN (100, 500, 900)"
step c2 300 python3 scripts/kexp.py range_in 30 \
  "SELECT COUNT(*), SUM(m) FROM synth WHERE $F2" \
  "SELECT COUNT(*) FROM synth WHERE $F2" \
  "SELECT COUNT(*) FROM synth WHERE r BETWEEN 114691 AND 344060" \
  "SELECT COUNT(*) FROM synth WHERE i IN (100, 500, 900)" \
  "SELECT SUM(m) FROM synth" \
  "SELECT SUM(m) FROM synth WHERE r BETWEEN 114691 AND 344060"
F3="(a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)"
step c3 300 python3 scripts/kexp.py bitmap5 30 \
  "SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE $F3" \
  "SELECT COUNT(*) FROM bitmap5 WHERE $F3" \
  "SELECT COUNT(*) FROM bitmap5 WHERE a = 10" \
  "SELECT COUNT(*) FROM bitmap5 WHERE a = 10 AND b IN (30, 70)" \
  "SELECT COUNT(*) FROM bitmap5 WHERE c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910" \
  "SELECT COUNT(*) FROM bitmap5 WHERE d <> 90" \
  "SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE a = 10"
