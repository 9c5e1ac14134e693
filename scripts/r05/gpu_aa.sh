#!/bin/bash
# Round 5: kernel-1 A/B of VGPR-reduced zero / equality tests in u256.cuh (ab/k1_a.so; C2 by
# scripts/ab_libs.py, and kernel 2's C4 on the same build), then the round-close suite + C4 SQ pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-aa}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 400 python3 -u scripts/ab_libs.py mythril_amd/libmythgpu.so ab/k1_a.so 4 > $OUT/ab_k1.log 2>&1 && \
AB_K2_MODES=scalar timeout -k 10 400 python3 -u scripts/ab_k2.py 2 ab/k1_a.so > $OUT/ab_k2.log 2>&1 && \
bash scripts/r05/gpu_y.sh $T
