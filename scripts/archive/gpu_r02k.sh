#!/bin/bash
# Kernel 2 in compiler form (folded selects, no copies): GPU suite + bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02k
mkdir -p $OUT
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== bench" && timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && \
echo "== k2 classes" && timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass.log 2>&1 && \
echo "== done"
