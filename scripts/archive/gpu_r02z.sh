#!/bin/bash
# Final tree check: GPU suite, smoke, two contexts after one-batch warm-ups, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${R02_OUT:-r02z}
mkdir -p $OUT
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
echo "== two ctx" && timeout -k 10 300 python -u scripts/two_ctx_check.py > $OUT/two_ctx.log 2>&1 && \
echo "== bench" && timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
echo "== done"
