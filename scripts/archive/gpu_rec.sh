#!/bin/bash
# Records change: lane + laser parity suites, then the C2 bench with records on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_laser.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_rec.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/bench_rec.log 2>&1
