#!/bin/bash
# Round 5: k_lane_step's HBM bytes per launch (FETCH_SIZE / WRITE_SIZE, separate passes) on
# the bench's profile command with the round-5 build, for bench.py's roofline.traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-k1}
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --unbucketed-steps 0 --profile-only"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- $B > $OUT/write.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1
