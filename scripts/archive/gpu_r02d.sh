#!/bin/bash
# LDS-resident kernel-1 runs + kernel-2 M=4: parity first, then interleaved A/Bs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_bench_fidelity.py tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_k.log 2>&1 &&
MG_BV_MPT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_m4.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_interleaved.py both > $OUT/ab.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
