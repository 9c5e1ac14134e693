#!/bin/bash
# Round 4: kernel-2 A/B on C4 (in-tree build against ab/ builds), results equal across builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-k}
mkdir -p $OUT
shift
AB_K2_MODES=scalar timeout -k 10 600 python -u scripts/ab_k2.py 3 "$@" > $OUT/ab_k2.log 2>&1
