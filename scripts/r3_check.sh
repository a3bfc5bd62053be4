#!/bin/bash
# Round-3 check on the GPU box: the GPU suite, then config 4 through bench.py (trim off, full-table parity).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
O=gpurun_out/r3check; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
fi
for wl in ${WLS:-groupby1m}; do
timeout -k 10 400 python -u bench.py --workload $wl --steps ${STEPS:-10} --warmup 2 --no-secondary --cpu-seconds 2 \
  > $O/bench_$wl.json 2> $O/bench_$wl.log || { echo "bench $wl failed rc=$?"; tail -20 $O/bench_$wl.log; exit 1; }
python - $O/bench_$wl.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["workload"], "ms/step %.3f kernel %.3f frac %.3f" % (d["ms_per_step"], d["roofline"]["kernel_ms_avg"], d["roofline"]["frac"]), "parity", d["parity_check"])
PY
done
