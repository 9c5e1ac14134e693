#!/bin/bash
# Round 4 close: k_sym_step FETCH_SIZE / WRITE_SIZE on the symbolic_lanes field's timed launches
# (scripts/r04/sym_timed.py, no profiling pass) with the final build, plus its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-au}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sym_trace -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py symbolic > $OUT/sym_trace.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py symbolic > $OUT/fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py symbolic > $OUT/write.log 2>&1
