#!/bin/bash
# Round 2: new parity tests first, then the full GPU suite, then one bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02a
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_k2_pinning.py tests/test_gpu_bench_fidelity.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
