#!/bin/bash
# Round 3 final evidence on the final tree: the -m gpu suite, smoke, the default
# bench line, its kernel trace, HBM passes of the bench's timed kernels (C2 +
# C4 -> traffic.json), k_sym_step HBM passes, and the LaserEVM host profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-f}
mkdir -p $OUT
P="python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --unbucketed-steps 0 --profile-only"
S="python3 -u scripts/r03/sym_lanes.py"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --unbucketed-steps 0 --profile-only > $OUT/prof_trace.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/bench_pmc/prof_fetch -o run --output-format csv -- $P > $OUT/bench_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/bench_pmc/prof_write -o run --output-format csv -- $P > $OUT/bench_write.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/sym_pmc/prof_fetch -o run --output-format csv -- $S > $OUT/sym_fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/sym_pmc/prof_write -o run --output-format csv -- $S > $OUT/sym_write.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-c4 --overlap-steps 0 --unbucketed-steps 0 \
    --large-steps 0 --no-cpu-baseline --no-roofline --symbolic-lanes 0 --taint-modes device \
    --host-profile $OUT/hostprof > $OUT/bench_host.json 2> $OUT/bench_host.err
