#!/bin/bash
# Round 6: k_lane_step and k_sym_step HBM bytes per launch on the round-6 build (FETCH_SIZE /
# WRITE_SIZE, one counter per run), then the host profiles of the in-situ fields.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-_p}
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --unbucketed-steps 0 --profile-only"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/k1_fetch -o run --output-format csv -- $B > $OUT/k1_fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/k1_write -o run --output-format csv -- $B > $OUT/k1_write.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/sym_fetch -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py symbolic code > $OUT/sym_fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/sym_write -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py symbolic code > $OUT/sym_write.log 2>&1 && \
bash scripts/r06/gpu_hostprof.sh ${1:-_p}
