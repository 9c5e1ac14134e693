#!/bin/bash
# Peaks probe, kernel-1 parity + laser tests, two C2 bench lines (no C4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 ./scripts/probes/peaks > $OUT/peaks.json 2> $OUT/peaks.err && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_laser.py -x -v --timeout 300 --timeout-method thread > $OUT/q_pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/q_bench1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/q_bench2.log 2>&1
