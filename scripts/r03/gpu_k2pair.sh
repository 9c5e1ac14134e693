#!/bin/bash
# Round 3: kernel-2 pair mode (two models per thread) -- parity, A/B against the
# single-model kernel, per-class timings; the symbolic-creation tests; the
# LaserEVM fields after the schedule change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_eval.py \
    tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py > $OUT/pytest_k2.log 2>&1 && \
AB_K2_MODES=scalar,pair timeout -k 10 600 python -u scripts/ab_k2.py 2 > $OUT/ab_k2_pair.log 2>&1 && \
MG_BV_PROG=pair timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass_pair.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbolic.py -k creation -v --timeout 240 --timeout-method thread > $OUT/pytest_creation.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-c4 --overlap-steps 0 --unbucketed-steps 0 \
    --large-steps 0 --no-cpu-baseline --no-roofline --symbolic-lanes 0 > $OUT/bench_fields.json 2> $OUT/bench_fields.err
