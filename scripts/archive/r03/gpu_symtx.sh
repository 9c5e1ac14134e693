#!/bin/bash
# Round 3: the symbolic_tx bench field alone (C2 minimal), after the symbolic GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
REPL=${2:-64}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbolic.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_sym.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-c4 --hooked-lanes 0 --taint-lanes 0 --overlap-steps 0 \
    --unbucketed-steps 0 --large-steps 0 --no-cpu-baseline --no-roofline --symbolic-replicas $REPL \
    > $OUT/bench_symtx.json 2> $OUT/bench_symtx.err
