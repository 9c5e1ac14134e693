#!/bin/bash
# Quick GPU iteration: kernel-1 parity tests + C2 bench only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_quick.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/bench_quick.log 2>&1
[ -n "$OPBENCH" ] && timeout -k 10 300 python -u scripts/opbench.py > $OUT/opbench.log 2>&1
true
