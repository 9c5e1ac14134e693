#!/bin/bash
# Kernel 2 with M models per thread: kernel-2 GPU tests at every M, then A/B of M = 1, 2, 4
# and of the previous build on C4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02p
mkdir -p $OUT
echo "== k2 tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_eval_mpt.py tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_k2.log 2>&1 && \
echo "== ab" && timeout -k 10 900 python -u scripts/ab_k2.py 3 ab/k2_old.so > $OUT/ab_k2.log 2>&1 && \
echo "== done"
