#!/bin/bash
# Round measurement on the GPU box: GPU tests, the default bench (config 5, 100 steps), the other workloads,
# then the rocprofv3 kernel-trace + PMC passes of the default bench.  Usage: round_bench.sh <tag>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
cd $R
bash scripts/gpu_check.sh tests || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench_adanalytics.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload range_in --steps 30 > gpurun_out/$TAG/bench_range_in.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload groupby1m --steps 5 --warmup 1 > gpurun_out/$TAG/bench_groupby1m.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload bitmap5 --steps 20 > gpurun_out/$TAG/bench_bitmap5.log 2>&1 || exit 1
bash scripts/profile_round.sh $TAG adanalytics
