#!/bin/bash
# C2 with two batches in flight (two library contexts / HIP streams) beside the
# one-stream figure, twice, plus a kernel trace of the two-stream run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02w
mkdir -p $OUT
B="python3 bench.py --no-c4 --hooked-lanes 0 --taint-lanes 0 --symbolic-calls 0 --no-cpu-baseline --large-steps 0 --unbucketed-steps 0 --no-roofline"
echo "== a" && timeout -k 10 300 $B --overlap-steps 20 > $OUT/a.json 2> $OUT/a.err && \
echo "== b" && timeout -k 10 300 $B --overlap-steps 40 > $OUT/b.json 2> $OUT/b.err && \
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- $B --steps 5 --overlap-steps 10 > $OUT/prof.log 2>&1 && \
echo "== done"
