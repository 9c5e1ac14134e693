#!/bin/bash
# GPU iteration: full parity suite + bench (no CPU baseline) + kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
echo "== pytest" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== bench" && timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 && \
echo "== trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --c4-steps 1 > $OUT/prof_trace.log 2>&1 && \
echo "== done"
