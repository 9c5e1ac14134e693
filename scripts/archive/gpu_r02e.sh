#!/bin/bash
# Kernel 2 with per-tile constant images: parity, then C4 A/B against the r01 kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_k2.log 2>&1 &&
MG_BV_MPT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_eval.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_k2_m1.log 2>&1 &&
MYTHGPU_LIB=$PWD/ab/lib_k2r01.so timeout -k 10 300 python -u scripts/ab_interleaved.py k2 1 > $OUT/ab_r01.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_interleaved.py k2 1,2,4 > $OUT/ab_new.log 2>&1 &&
MYTHGPU_LIB=$PWD/ab/lib_k2r01.so timeout -k 10 300 python -u scripts/ab_interleaved.py k2 1 > $OUT/ab_r01_again.log 2>&1
