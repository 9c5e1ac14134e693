#!/bin/bash
# Round 5: A/B of compiler scheduling options for the whole library (ab/f_ilp.so:
# -amdgpu-sched-strategy=max-ilp; ab/f_bias0.so: -amdgpu-schedule-metric-bias=0) on C2 and C4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-ae}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 400 python3 -u scripts/ab_libs.py mythril_amd/libmythgpu.so ab/f_ilp.so ab/f_bias0.so 6 > $OUT/ab_k1.log 2>&1
