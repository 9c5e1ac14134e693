#!/bin/bash
# Round 5: k_sym_step WRITE_SIZE with every lane stopped after K steps (K = 0 1 3 5): the
# per-launch write floor and the slope per lane-step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-s}
mkdir -p $OUT
for k in 0 1 3 5; do
  MG_SYM_MAXSTEPS=$k timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/w$k -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py symbolic code > $OUT/w$k.log 2>&1 || exit 1
done
