#!/bin/bash
# Round 6 close-out: the -m gpu suite, the smoke, the default bench line (full record kept), then
# the same bench command under rocprofv3 --kernel-trace --stats (the per-kernel averages the
# roofline fields must agree with).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-_f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py --full-record $OUT/bench_full.json > $OUT/bench.log 2>&1 && \
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- \
    python3 -u bench.py --full-record $OUT/bench_trace_full.json > $OUT/bench_trace.log 2>&1
