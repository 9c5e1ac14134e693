#!/bin/bash
# Round 5: A/B of kernel 2's division with 64-bit funnel shifts in the normalisation
# (V28): C4, C2, and the division / numerics tests on V27.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-af}
OUT=gpurun_out/r05$T
mkdir -p $OUT
AB_K2_MODES=scalar timeout -k 10 500 python3 -u scripts/ab_k2.py 3 ab/k2_v28.so > $OUT/ab_k2.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/ab_libs.py mythril_amd/libmythgpu.so ab/k2_v28.so 3 > $OUT/ab_k1.log 2>&1 && \
MYTHGPU_LIB=$PWD/ab/k2_v28.so timeout -k 10 400 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_lanes.py tests/test_gpu_solver.py -v --timeout 240 --timeout-method thread > $OUT/pytest_v28.log 2>&1
