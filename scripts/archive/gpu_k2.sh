#!/bin/bash
# Kernel-2 parity tests + per-op-class timing (scripts/k2_opclass.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > $OUT/k2_pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass.log 2>&1
