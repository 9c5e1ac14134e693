#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 600 python -u scripts/r03/prof_fields.py $OUT/hostprof ${2:-4096} ${3:-hooked,taint} > $OUT/prof_fields.log 2>&1
