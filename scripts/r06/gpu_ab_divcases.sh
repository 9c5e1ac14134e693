#!/bin/bash
# Round 6: interleaved A/B of the exact procedure's pinned-divisor case split on the in-situ fields.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-_abd}
mkdir -p $OUT
timeout -k 10 1000 python -u scripts/r06/ab_rel.py $OUT/ab_divcases.json 2 MYTHSMT_DIVCASES 0,1 \
    overflow.sol.o,exceptions.sol.o,flag_array.sol.o > $OUT/ab_divcases.log 2>&1
