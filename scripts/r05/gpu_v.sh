#!/bin/bash
# Round 5: the -m gpu suite on kernel 2's hot-op-bit build (V14, in-tree), the A/B of two
# further dispatch variants against it, and the C4 SQ pass of the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-v}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
AB_K2_MODES=scalar timeout -k 10 700 python3 -u scripts/ab_k2.py 3 ab/k2_v15.so ab/k2_v16.so > $OUT/ab_k2.log 2>&1 && \
bash scripts/r05/gpu_k2c4sq.sh $T
