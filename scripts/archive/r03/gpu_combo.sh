#!/bin/bash
# Round 3: selected GPU tests, then the LaserEVM bench fields with host profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_bridge.py tests/test_gpu_symbolic.py tests/test_gpu_solver.py} \
    -x -q --timeout 200 --timeout-method thread > $OUT/pytest_sel.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --no-c4 --overlap-steps 0 --unbucketed-steps 0 \
    --large-steps 0 --no-cpu-baseline --no-roofline --symbolic-replicas ${2:-8} \
    --host-profile $OUT/hostprof > $OUT/bench_host.json 2> $OUT/bench_host.err
