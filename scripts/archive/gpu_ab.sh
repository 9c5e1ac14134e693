#!/bin/bash
# A/B of kernel-2 program-fetch variants after the parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
echo "== pytest" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== bench scalar" && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 && \
echo "== bench scalar-prog" && MG_BV_PROG=scalar timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_lds.log 2>&1 && \
echo "== done"
