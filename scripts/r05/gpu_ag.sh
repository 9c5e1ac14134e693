#!/bin/bash
# Round 5: host profile of the myth_analyze field on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-ag}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 300 python -u scripts/r05/prof_analyze.py $OUT/hostprof_analyze.txt > $OUT/hostprof_analyze.log 2>&1
