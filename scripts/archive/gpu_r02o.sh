#!/bin/bash
# Keccak rotations as alignbit pairs: GPU suite on the new build, then A/B of the two builds
# (and of the wave-aligned lane order) on C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02o
mkdir -p $OUT
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== ab" && timeout -k 10 600 python -u scripts/ab_libs.py ab/rot_old.so ab/rot_new.so ab/rot_new.so:wave 4 > $OUT/ab_rot.log 2>&1 && \
echo "== done"
