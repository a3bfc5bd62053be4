#!/bin/bash
# GPU suite, then kernel traces of the secondary workloads and PMC passes (config 4: FETCH / WRITE / LDS bank
# conflicts; configs 2 and 3: FETCH / WRITE) for the round profile.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
SKIP_TESTS=${SKIP_TESTS:-0} WLS="${CHECK_WLS:-bitmap5}" STEPS=20 bash scripts/r3_check.sh || exit 1
WLS="range_in bitmap5 groupby1m groupby1m_zipf adanalytics_inv" PMC_WLS="groupby1m range_in bitmap5" \
  PMC_COUNTERS="FETCH_SIZE WRITE_SIZE SQ_LDS_BANK_CONFLICT" bash scripts/r3_prof.sh ${TAG:-r3c} || exit 1
