#!/bin/bash
# Kernel-1 A/B: C2 bench with ab/base.so and the in-tree library (records off / on), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4"
for i in 1 2; do
  MYTHGPU_LIB=ab/base.so timeout -k 10 300 $B --rec-cap 0 > $OUT/ab_base_$i.log 2>&1 && \
  timeout -k 10 300 $B --rec-cap 0 > $OUT/ab_new0_$i.log 2>&1 && \
  timeout -k 10 300 $B --rec-cap 128 > $OUT/ab_new_$i.log 2>&1 || exit 1
done
