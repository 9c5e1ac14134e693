#!/bin/bash
# Round 4: does a field run before symbolic_tx change its wall time?  symbolic_tx alone, then
# after the symbolic/taint lane fields, then after the hooked/taint C2 fields.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-x}
mkdir -p $OUT
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c4 --overlap-steps 0 --unbucketed-steps 0 --large-steps 0 --analyses 0"
timeout -k 10 300 $B --hooked-lanes 0 --taint-lanes 0 --symbolic-lanes 0 > $OUT/alone.json 2> $OUT/alone.err && \
timeout -k 10 300 $B --hooked-lanes 0 --taint-lanes 0 > $OUT/after_lanes.json 2> $OUT/after_lanes.err && \
timeout -k 10 300 $B --symbolic-lanes 0 > $OUT/after_c2host.json 2> $OUT/after_c2host.err
