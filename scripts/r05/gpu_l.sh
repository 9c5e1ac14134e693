#!/bin/bash
# Round 5: kernel-2 numerics on the in-tree build, the kernel-2 A/B (in-tree vs ab/k2_*.so, C4,
# interleaved rounds, identical results), then the k_sym_step write experiment.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-l}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py -v --timeout 240 --timeout-method thread > $OUT/pytest_k2.log 2>&1 && \
AB_K2_MODES=scalar timeout -k 10 600 python3 -u scripts/ab_k2.py 3 ${AB_LIBS:-ab/k2_base.so ab/k2_v3.so} > $OUT/ab_k2.log 2>&1 && \
bash scripts/r05/gpu_symflush.sh $T
