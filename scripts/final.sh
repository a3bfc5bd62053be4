#!/bin/bash
# Closing check on the GPU box: the whole -m gpu suite, then the default bench run (N = 1, headline +
# secondary workloads with CPU baselines and full-size parity).  Stops after a failed test run.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$R"
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?
echo "bench rc=$rc"; grep '"metric"' "$OUT/bench.log" | tail -1 | cut -c1-400
exit $rc
