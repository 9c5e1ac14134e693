#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-q}
OUT=gpurun_out/r05$T
mkdir -p $OUT
AB_K2_MODES=scalar timeout -k 10 700 python3 -u scripts/ab_k2.py 3 ${AB_LIBS} > $OUT/ab_k2.log 2>&1
