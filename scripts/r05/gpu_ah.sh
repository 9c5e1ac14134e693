#!/bin/bash
# Round 5: kernel-2 A/B of the blocks-per-launch target (BV_GROUP_TARGET 8192 / 2048 against 4096).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-ah}
OUT=gpurun_out/r05$T
mkdir -p $OUT
AB_K2_MODES=scalar timeout -k 10 500 python3 -u scripts/ab_k2.py 3 ab/k2_g8192.so ab/k2_g2048.so > $OUT/ab_k2.log 2>&1
