#!/bin/bash
# Kernel-1 clock bins (diagnostic build ab/clk.so: dispatch head / handler / fetch)
# for the LDS-resident and register run forms; kernel-2 suite on the restored kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02f
mkdir -p $OUT
MG_K1_RUNS=lds timeout -k 10 200 python -u scripts/k1_clocks.py > $OUT/clk_lds.log 2>&1 &&
MG_K1_RUNS=reg timeout -k 10 200 python -u scripts/k1_clocks.py > $OUT/clk_reg.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_k2.log 2>&1
