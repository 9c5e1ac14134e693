#!/bin/bash
# Round 5: round-close suite on the byte-offset kernel-2 build (tests, smoke, bench, bench under
# rocprofv3 --kernel-trace --stats), then kernel 2's C4 SQ pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-y}
OUT=gpurun_out/r05$T
mkdir -p $OUT
bash scripts/r05/gpu_suite_prof.sh $T && \
bash scripts/r05/gpu_k2c4sq.sh $T
