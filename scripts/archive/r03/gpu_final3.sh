#!/bin/bash
# Round 3 final: suite, smoke, default bench line and host profiles after the
# fast-path fix (kernels unchanged since r03f: its trace and PMC passes stand).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-g}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-c4 --overlap-steps 0 --unbucketed-steps 0 \
    --large-steps 0 --no-cpu-baseline --no-roofline --symbolic-lanes 0 --taint-modes device \
    --host-profile $OUT/hostprof > $OUT/bench_host.json 2> $OUT/bench_host.err
