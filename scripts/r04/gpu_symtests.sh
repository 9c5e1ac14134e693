#!/bin/bash
# Round 4: the symbolic GPU tests and the co-simulation's escaped opcodes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-m}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_symbolic.py tests/test_gpu_integration.py tests/test_gpu_fork_filter.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest_sym.log 2>&1 && \
timeout -k 10 300 python -u scripts/r04/sym_escapes.py > $OUT/sym_escapes.log 2>&1
