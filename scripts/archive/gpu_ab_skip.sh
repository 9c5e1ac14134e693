#!/bin/bash
# A/B: default structurizer vs -structurizecfg-skip-uniform-regions (ab/libmythgpu_skip.so):
# GPU parity suite on the variant, kernel-2 op classes and C2/C4 bench lines for both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
V=$PWD/ab/libmythgpu_skip.so
echo "== pytest variant" && MYTHGPU_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/ab_pytest.log 2>&1 && \
echo "== k2 base" && timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/ab_k2_base.log 2>&1 && \
echo "== k2 variant" && MYTHGPU_LIB=$V timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/ab_k2_var.log 2>&1 && \
echo "== bench base" && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/ab_bench_base.log 2>&1 && \
echo "== bench variant" && MYTHGPU_LIB=$V timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/ab_bench_var.log 2>&1 && \
echo "== done"
