#!/bin/bash
# Sweep the direct kernel's per-CU workgroups and LDS slots per wave on the default bench (config 5).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/sweep; mkdir -p "$OUT"
for wgs in ${WGS_LIST:-3 4 5 6 8}; do
  for slots in ${SLOTS_LIST:-0 3 4 6}; do
    PGPU_DIRECT_WGS=$wgs PGPU_DIRECT_SLOTS=$slots timeout -k 10 120 python3 "$R/bench.py" --steps 50 --warmup 5 \
      --no-cpu-baseline --no-check > "$OUT/w${wgs}_s${slots}.log" 2>&1 || { echo "fail wgs=$wgs slots=$slots rc=$?"; exit 1; }
    echo "wgs=$wgs slots=$slots $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' "$OUT/w${wgs}_s${slots}.log" | tr '\n' ' ')"
  done
done
