#!/bin/bash
# Round 3: symbolic-lane co-simulation first, then the whole GPU parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_symbolic.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_sym.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
