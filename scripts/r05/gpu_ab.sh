#!/bin/bash
# Round 5: A/B of the fp64-derived Moller-Granlund reciprocal in u256.cuh (ab/k2_v24.so) on C4
# (kernel 2's division sites) and C2 (kernel 1), then kernel 2's numerics tests on that build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-ab}
OUT=gpurun_out/r05$T
mkdir -p $OUT
AB_K2_MODES=scalar timeout -k 10 500 python3 -u scripts/ab_k2.py 3 ab/k2_v24.so > $OUT/ab_k2.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/ab_libs.py mythril_amd/libmythgpu.so ab/k2_v24.so 3 > $OUT/ab_k1.log 2>&1 && \
MYTHGPU_LIB=$PWD/ab/k2_v24.so timeout -k 10 400 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_lanes.py -v --timeout 240 --timeout-method thread > $OUT/pytest_v24.log 2>&1
