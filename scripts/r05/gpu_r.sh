#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_fork_filter.py tests/test_gpu_solver.py -v --timeout 240 --timeout-method thread > $OUT/pytest_k2.log 2>&1 && \
bash scripts/r05/gpu_k2c4sq.sh $T && \
bash scripts/r05/gpu_symsteps.sh $T
