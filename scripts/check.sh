#!/bin/bash
# GPU check: the parity suites touched this round, then rocprof kernel stats of the bench workloads named in
# $WLS (default: the sliced-aggregation ones).  Usage: check.sh <tag>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_mv_columns.py tests/test_gpu_full_size.py tests/test_gpu_segment_stats.py} \
  -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"
# a failed or faulted test run ends the GPU work of this call (rc 5: no tests selected is fine)
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --no-cpu-baseline --no-check --no-secondary"
for wl in ${WLS:-range_in bitmap5 adanalytics_exact}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$wl" -o run -- \
    python3 $BENCH --workload $wl --steps ${STEPS:-10} --warmup 2 > "$OUT/$wl.log" 2>&1 || { echo "trace $wl failed rc=$?"; tail -5 "$OUT/$wl.log"; exit 1; }
  grep -h '"metric"' "$OUT/$wl.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_avg'],3), round(d['roofline']['frac'],3))"
done
echo done
