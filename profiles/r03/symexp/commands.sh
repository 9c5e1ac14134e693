#!/bin/bash
# Round 3: symbolic EXP on the device -- the symbolic co-simulation tests first,
# then the suite, smoke and the default bench line (symbolic_tx escapes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-j}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_symbolic.py > $OUT/pytest_sym.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
