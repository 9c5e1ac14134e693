#!/bin/bash
# Round 6: interleaved A/B of the exact procedure's cone-first phase on the in-situ fields.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-_ab}
mkdir -p $OUT
timeout -k 10 900 python -u scripts/r06/ab_rel.py $OUT/ab_rel.json 2 > $OUT/ab_rel.log 2>&1
