#!/bin/bash
# GPU-box check sequence: each GPU step under its own time limit; stop at the first crash/timeout
# (test failures, exit 1, do not stop the sequence).  Logs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -u __graft_entry__.py smoke ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    bench) run bench 600 python -u bench.py --steps 10 --warmup 2 ;;
    bench_range) run bench_range 600 python -u bench.py --steps 10 --warmup 2 --workload range_in ;;
    bench_gb) run bench_gb 600 python -u bench.py --steps 5 --warmup 1 --workload groupby1m ;;
    bench_bm) run bench_bm 600 python -u bench.py --steps 10 --warmup 2 --workload bitmap5 ;;
    round_prof) run round_prof 900 bash scripts/profile_round.sh "${PROF_TAG:-prof}" ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check ;;
  esac
done
