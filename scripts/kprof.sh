#!/bin/bash
# Phase profile (PGPU_PROFILE=1) of a few adanalytics shapes; output gpurun_out/kprof.log
mkdir -p gpurun_out
T=adAnalytics
PGPU_PROFILE=1 timeout -k 10 200 python -u scripts/kexp.py adanalytics 30 \
 "SELECT COUNT(*) FROM $T" \
 "SELECT COUNT(*) FROM $T WHERE daysSinceEpoch BETWEEN 17849 AND 17856" \
 "SELECT SUM(clicks) FROM $T" \
 "$@" > gpurun_out/kprof.log 2>&1
