#!/bin/bash
# Round 5: the whole -m gpu suite on the build with k_sym_step's argument structs out of scratch
# and kernel 2's combined epilogue test, then k_sym_step's PMC passes, kernel 2's C4 SQ pass and
# the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-t}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
bash scripts/r05/gpu_sympmc.sh $T code && \
bash scripts/r05/gpu_k2c4sq.sh $T && \
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
