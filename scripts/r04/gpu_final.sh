#!/bin/bash
# Round 4 close: the -m gpu suite, smoke, the default bench line, and the kernel trace of the
# bench command (C2 + C4 launches) whose averages the bench's HIP-event timings must match.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o run --output-format csv -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --hooked-lanes 0 --overlap-steps 0 --unbucketed-steps 0 --large-steps 0 --taint-lanes 0 --symbolic-lanes 0 --symbolic-replicas 0 --analyses 0 > $OUT/bench_trace.log 2>&1
