#!/bin/bash
# Kernel 1: merged decode/run fetch + runs closed by a jump. Parity, A/B, clock bins.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_interleaved.py k1 > $OUT/ab_k1.log 2>&1 &&
MG_K1_RUNS=lds timeout -k 10 200 python -u scripts/k1_clocks.py > $OUT/clk_lds.log 2>&1
