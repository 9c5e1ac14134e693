#!/bin/bash
# Round 3: host profiles (cProfile) of the LaserEVM bench fields on the GPU box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --no-c4 --overlap-steps 0 --unbucketed-steps 0 \
    --large-steps 0 --no-cpu-baseline --no-roofline --symbolic-replicas ${2:-8} ${3:-} \
    --host-profile $OUT/hostprof > $OUT/bench_host.json 2> $OUT/bench_host.err
