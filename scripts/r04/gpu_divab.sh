#!/bin/bash
# Round 4: kernel-2 division variants (ab/div_*.so, -DMG_DIV_SKIP / -DMG_DIV_SS_MAX): the
# kernel-2 numerics tests on each variant, then the C4 A/B against the in-tree build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-ad}
mkdir -p $OUT
for v in div_skip div_ss8 div_ss0; do
  MYTHGPU_LIB=ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_$v.log 2>&1 || exit 1
done
AB_K2_MODES=scalar timeout -k 10 600 python -u scripts/ab_k2.py 3 ab/div_skip.so ab/div_ss8.so ab/div_ss0.so > $OUT/ab_k2.log 2>&1
