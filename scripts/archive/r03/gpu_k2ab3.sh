#!/bin/bash
# Kernel 2 A/B, third pass: operand A loaded into the accumulator's registers
# (the flattener keeps the accumulator in position A: swapped compares, bvrsub,
# rconcat) against the previous round-3 build (ab/k2_r03.so) and round 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-u}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py > $OUT/pytest_k2.log 2>&1 && \
timeout -k 10 600 python -u scripts/ab_k2.py 2 ab/k2_r03.so:legacy ab/k2_old.so:legacy > $OUT/ab_k2.log 2>&1 && \
timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass.log 2>&1
