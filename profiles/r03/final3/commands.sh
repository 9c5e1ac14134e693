#!/bin/bash
# Round 3 final: kernel-2 uniform shifts (parity, A/B vs ab/k2_dmajor.so, class
# timings), host A/B in one process, suite, smoke, default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-i}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_eval.py \
    tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py > $OUT/pytest_k2.log 2>&1 && \
AB_K2_MODES=scalar timeout -k 10 600 python -u scripts/ab_k2.py 2 ab/k2_dmajor.so > $OUT/ab_k2_ushift.log 2>&1 && \
timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass_ushift.log 2>&1 && \
timeout -k 10 600 python -u scripts/r03/host_ab.py > $OUT/host_ab.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
