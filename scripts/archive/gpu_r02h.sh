#!/bin/bash
# Full bench line (C2 + hooked C2 + C4) on the current tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02h
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
