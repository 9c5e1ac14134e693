#!/bin/bash
# Kernel-2 superinstructions (bv_fuse): parity (fused vs unfused vs oracle), C4
# A/B all shapes, two shapes and unfused in one library, op-class timings, then the GPU suite,
# smoke and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-f}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_eval.py \
    tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py > $OUT/pytest_k2.log 2>&1 && \
AB_K2_MODES=scalar,scalar-fuse2,scalar-fuse1,scalar-fuse0 timeout -k 10 600 python -u scripts/ab_k2.py 2 > $OUT/ab_k2_fuse.log 2>&1 && \
timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass_fuse.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
