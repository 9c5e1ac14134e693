#!/bin/bash
# In-place capacity regrow on the GPU, then the LaserEVM / taint GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02v
mkdir -p $OUT
echo "== regrow" && timeout -k 10 600 python -u -m pytest tests/test_gpu_regrow.py tests/test_gpu_taint.py tests/test_gpu_laser.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_regrow.log 2>&1 && \
echo "== done"
