#!/bin/bash
# Round 5: k_sym_step WRITE_SIZE with and without an evicting read between upload and launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-k}
mkdir -p $OUT
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/sym_write_plain -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py symbolic code > $OUT/plain.log 2>&1 && \
MG_SYM_FLUSH=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/sym_write_flush -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py symbolic code > $OUT/flush.log 2>&1
