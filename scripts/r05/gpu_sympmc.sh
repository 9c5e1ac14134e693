#!/bin/bash
# Round 5: k_sym_step FETCH_SIZE / WRITE_SIZE on the symbolic_lanes and taint_lanes fields'
# timed launches (scripts/r04/sym_timed.py, no profiling pass), each pass its own run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-s}
mkdir -p $OUT
ORDERS=${2:-code}
for order in $ORDERS; do
for kind in symbolic taint; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/${kind}_${order}_fetch -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py $kind $order > $OUT/${kind}_${order}_fetch.log 2>&1 && \
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/${kind}_${order}_write -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py $kind $order > $OUT/${kind}_${order}_write.log 2>&1 || exit 1
done
done
