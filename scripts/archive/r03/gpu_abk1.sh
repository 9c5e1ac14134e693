#!/bin/bash
# Kernel 1 C2: the round-2 library build (ab/k2_old.so) against the in-tree one,
# alternating processes (scripts/ab_libs.py): is the C2 difference the library?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-r}
mkdir -p $OUT
timeout -k 10 500 python -u scripts/ab_libs.py ab/k2_old.so mythril_amd/libmythgpu.so 4 > $OUT/ab_k1.log 2>&1
