#!/bin/bash
# Round 6: the -m gpu suite, the smoke and the default bench line, as the driver runs them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 1000 python -u bench.py --full-record $OUT/bench_full.json > $OUT/bench.log 2>&1
