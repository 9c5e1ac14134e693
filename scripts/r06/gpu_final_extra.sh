#!/bin/bash
# Round 6: BECToken -t 2 and the in-situ host profiles on the final build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-_x}
mkdir -p $OUT
timeout -k 10 400 python -u scripts/r06/c3_bec.py 2 > $OUT/c3_bec2_gpu.log 2>&1 && \
bash scripts/r06/gpu_hostprof.sh ${1:-_x}
