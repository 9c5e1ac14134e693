#!/bin/bash
# Round 5: host profile of the myth_analyze field, then the round-close suite (tests, smoke, bench,
# bench under rocprofv3 --kernel-trace --stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-w}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 300 python -u scripts/r05/prof_analyze.py $OUT/hostprof_analyze.txt > $OUT/hostprof_analyze.log 2>&1 && \
bash scripts/r05/gpu_suite_prof.sh $T
