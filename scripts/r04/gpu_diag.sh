#!/bin/bash
# Round 4: the symbolic_tx host profile, then the symbolic co-simulation's escaped opcodes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-l}
mkdir -p $OUT
bash scripts/r04/gpu_hostprof.sh ${1:-l} && \
timeout -k 10 300 python -u scripts/r04/sym_escapes.py > $OUT/sym_escapes.log 2>&1
