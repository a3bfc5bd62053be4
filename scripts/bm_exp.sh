#!/bin/bash
# bitmap5 (config 3) breakdown: leaf-type variants + phase profile
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out
Q="SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE (a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)"
timeout -k 10 300 python3 $R/scripts/kexp.py bitmap5 30 "$Q" \
  "SELECT COUNT(*) FROM bitmap5 WHERE (a = 10 AND b IN (30, 70)) OR (c = 50 AND d <> 90 AND e BETWEEN 640 AND 1910)" \
  "SELECT COUNT(*) FROM bitmap5 WHERE a = 10" "SELECT COUNT(*) FROM bitmap5 WHERE b IN (30, 70)" \
  "SELECT COUNT(*) FROM bitmap5 WHERE c = 50" "SELECT COUNT(*) FROM bitmap5 WHERE d <> 90" \
  "SELECT COUNT(*) FROM bitmap5 WHERE e BETWEEN 640 AND 1910" "SELECT SUM(m1), SUM(m2) FROM bitmap5 WHERE c = 50" \
  > $R/gpurun_out/bm_variants.log 2>&1 || exit 1
grep " ms " $R/gpurun_out/bm_variants.log
