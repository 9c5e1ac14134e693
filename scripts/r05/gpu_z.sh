#!/bin/bash
# Round 5: kernel-2 A/B of the constant byte offset with (V20) and without (V20b) the slot column, and the VALU eq/zero tests on each (V21, V22) against the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-z}
OUT=gpurun_out/r05$T
mkdir -p $OUT
AB_K2_MODES=scalar timeout -k 10 600 python3 -u scripts/ab_k2.py 3 ab/k2_v20.so ab/k2_v20b.so ab/k2_v21.so ab/k2_v22.so > $OUT/ab_k2.log 2>&1
