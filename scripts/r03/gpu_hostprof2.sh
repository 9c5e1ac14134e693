#!/bin/bash
# Round 3: cProfile of the LaserEVM fields (hooked_c2, taint_c2 device mode,
# symbolic_tx) after the host-path changes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-c4 --overlap-steps 0 --unbucketed-steps 0 \
    --large-steps 0 --no-cpu-baseline --no-roofline --symbolic-lanes 0 --taint-modes device \
    --host-profile $OUT/hostprof > $OUT/bench_host.json 2> $OUT/bench_host.err
