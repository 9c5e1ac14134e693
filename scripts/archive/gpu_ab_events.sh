#!/bin/bash
# A/B: per-batch timing events between the C2 launches vs one event pair (MG_BATCH_EVENTS=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/abe_on_$r.log 2>&1 || exit 1
  MG_BATCH_EVENTS=0 timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/abe_off_$r.log 2>&1 || exit 1
done
