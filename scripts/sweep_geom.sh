#!/bin/bash
# Direct-kernel geometry sweep (LDS slots per wave x workgroups per CU) on configs 2 and 3 through bench.py:
# gpurun_out/sweep_geom.log
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R; mkdir -p gpurun_out; : > gpurun_out/sweep_geom.log
for wl in ${WLS:-range_in bitmap5}; do
  for cfg in ${SWEEP:-"0 0" "2 4" "4 4" "6 4" "3 3" "3 2"}; do
    set -- $cfg
    env $( [ "$1" != 0 ] && echo PGPU_DIRECT_SLOTS=$1 ) $( [ "$2" != 0 ] && echo PGPU_DIRECT_WGS=$2 ) PGPU_BENCH_DUMMY=1 \
      timeout -k 10 200 python3 -u bench.py --workload $wl --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --no-check \
      > gpurun_out/sg.json 2> gpurun_out/sg.log || { echo "$wl $cfg failed"; tail -5 gpurun_out/sg.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/sg.json').read().strip().splitlines()[-1])
print('$wl slots/wgs $cfg', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms_avg'],3), round(d['roofline']['frac'],3))" >> gpurun_out/sweep_geom.log
  done
done
cat gpurun_out/sweep_geom.log
