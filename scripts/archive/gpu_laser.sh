#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_laser.py tests/test_gpu_lanes.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_laser.log 2>&1
