#!/bin/bash
# Round 4: symbolic and taint GPU tests, the co-simulation's escapes, and the analyses field alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-ai}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_symbolic.py tests/test_gpu_taint.py tests/test_gpu_integration.py tests/test_gpu_fork_filter.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/r04/sym_escapes.py > $OUT/sym_escapes.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-c4 --hooked-lanes 0 --overlap-steps 0 --unbucketed-steps 0 --large-steps 0 --taint-lanes 0 --symbolic-lanes 0 --symbolic-replicas 0 --analyses 2 > $OUT/analyses.json 2> $OUT/analyses.err
