#!/bin/bash
# Zipf(1.1) config 4 with and without the frame-of-reference phase 2: kernel split by rocprof.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
Q4="SELECT k, SUM(m), MAX(m), COUNT(*) FROM synth GROUP BY k ORDER BY SUM(m) DESC LIMIT 100"
for F in 0 1; do
  OUT=$R/gpurun_out/r2exp10/for$F; mkdir -p $OUT
  PGPU_NO_FOR=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 $R/scripts/kexp.py groupby1m_zipf 60 "$Q4" > $OUT/log 2>&1 || { echo "rc=$?"; tail -5 $OUT/log; exit 1; }
  echo "== PGPU_NO_FOR=$F"; grep " ms " $OUT/log | cut -c1-60; grep "part_" $OUT/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-120
done
