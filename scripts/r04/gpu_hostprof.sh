#!/bin/bash
# Round 4: symbolic_tx alone under cProfile (host-time work).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-d}
mkdir -p $OUT/hostprof
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c4 --hooked-lanes 0 --overlap-steps 0 \
    --unbucketed-steps 0 --large-steps 0 --taint-lanes 0 --symbolic-lanes 0 > $OUT/bench_symtx.json 2> $OUT/bench_symtx.err && \
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c4 --hooked-lanes 0 --overlap-steps 0 \
    --unbucketed-steps 0 --large-steps 0 --taint-lanes 0 --symbolic-lanes 0 --host-profile $OUT/hostprof \
    > $OUT/bench_symtx_prof.json 2> $OUT/bench_symtx_prof.err
