#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-o}
OUT=gpurun_out/r05$T
mkdir -p $OUT
bash scripts/r05/gpu_k2c4sq.sh $T && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
