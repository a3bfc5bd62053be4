#!/bin/bash
# Round-2 measurement: the default bench (config 5 headline + configs 2-4 and variants), then the rocprofv3
# kernel-trace / PMC passes of config 5.  Usage: round_r2.sh <tag>
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1
cd $R
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u bench.py > gpurun_out/$TAG/bench_default.log 2>&1 || { echo "bench failed rc=$?"; exit 1; }
tail -c 400 gpurun_out/$TAG/bench_default.log
bash scripts/profile_round.sh $TAG adanalytics
