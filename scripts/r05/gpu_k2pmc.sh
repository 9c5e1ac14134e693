#!/bin/bash
# Round 5: k_bv_eval's HBM bytes per C4 launch (FETCH_SIZE / WRITE_SIZE, separate passes) on the
# round-5 build, for the constraint_evals line's roofline.traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-k2p}
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- python3 -u scripts/r03/k2_c4.py > $OUT/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- python3 -u scripts/r03/k2_c4.py > $OUT/write.log 2>&1
