#!/bin/bash
# Round 5: GPU tests touched by the k_sym_step changes, then the symbolic PMC and kernel-2 SQ passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-h}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_integration.py tests/test_gpu_taint.py tests/test_gpu_symbolic.py tests/test_gpu_lanes.py -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 && \
bash scripts/r05/gpu_sympmc.sh $T && \
bash scripts/r05/gpu_k2sq.sh $T
