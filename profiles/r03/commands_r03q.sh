#!/bin/bash
# Round 3: the default bench line, its kernel trace, and the host profiles of
# the LaserEVM fields.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err && \
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-c4 --overlap-steps 0 --unbucketed-steps 0 \
    --large-steps 0 --no-cpu-baseline --no-roofline --symbolic-lanes 0 \
    --host-profile $OUT/hostprof > $OUT/bench_host.json 2> $OUT/bench_host.err && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/twoctx -o run -- python3 -u scripts/two_ctx_check.py > $OUT/twoctx.log 2>&1
