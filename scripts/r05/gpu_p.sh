#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-p}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 400 python3 -u scripts/r05/ab_lpw.py > $OUT/ab_lpw.log 2>&1
