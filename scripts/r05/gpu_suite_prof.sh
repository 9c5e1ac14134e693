#!/bin/bash
# Round 5: the -m gpu suite, the smoke, the default bench line, then the same bench command under
# rocprofv3 --kernel-trace --stats (the per-kernel averages the roofline fields must agree with).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-n}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 ; \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 -u bench.py > $OUT/bench_trace.log 2>&1
