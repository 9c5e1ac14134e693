#!/bin/bash
# Round 4: several measurements in one box: symbolic_tx host profile, a kernel-2 A/B
# against the given library builds, then the round-close suite + bench + bench trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-t}
shift
bash scripts/r04/gpu_hostprof.sh $TAG && \
bash scripts/r04/gpu_k2ab.sh $TAG "$@" && \
bash scripts/r04/gpu_final.sh $TAG
