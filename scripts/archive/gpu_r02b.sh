#!/bin/bash
# Round 2: new parity tests, kernel-2 models-per-thread A/B, full GPU suite, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_k2_pinning.py tests/test_gpu_eval.py tests/test_gpu_bench_fidelity.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 &&
for m in 1 2 4; do MG_BV_MPT=$m timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_mpt$m.log 2>&1 || exit 1; done &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
