#!/bin/bash
# One GPU-box pass: the named test files (TESTS, default the whole -m gpu suite), then the default bench line and,
# with NODE=1, the headline through the in-process node path.  Usage: round.sh <tag>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$R"
timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"
# assertion failures (1) still let the bench run; a fault, abort, time limit or pytest error ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
TRC=$rc
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --full-out "$OUT/bench_full.json" ${BENCH_ARGS:-} > "$OUT/bench.out" 2> "$OUT/bench.err"
  rc=$?
  echo "bench rc=$rc"; wc -c "$OUT/bench.out"; tail -c 600 "$OUT/bench.out"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/bench.err"; exit $rc; fi
fi
if [ "${NODE:-0}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --node --gpus 1 --no-secondary --steps 300 --full-out "$OUT/node_full.json" > "$OUT/node.out" 2> "$OUT/node.err"
  rc=$?
  echo "node rc=$rc"; tail -c 400 "$OUT/node.out"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/node.err"; exit $rc; fi
fi
echo "done (tests rc=$TRC)"
