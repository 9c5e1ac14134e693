#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02m
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbolic.py -v --timeout 240 --timeout-method thread > $OUT/pytest_sym.log 2>&1
