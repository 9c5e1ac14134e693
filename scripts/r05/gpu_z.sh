#!/bin/bash
# Round 5: kernel-2 A/B of the per-lane slot column (V19) and the constant byte offset (V20) against the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-z}
OUT=gpurun_out/r05$T
mkdir -p $OUT
AB_K2_MODES=scalar timeout -k 10 600 python3 -u scripts/ab_k2.py 3 ab/k2_v19.so ab/k2_v20.so > $OUT/ab_k2.log 2>&1
