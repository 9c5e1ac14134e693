#!/bin/bash
# Symbolic lanes: co-simulation + end-to-end tests, then the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02l
mkdir -p $OUT
echo "== symbolic" && timeout -k 10 300 python -u -m pytest tests/test_gpu_symbolic.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest_sym.log 2>&1 ; \
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 ; \
echo "== done"
