#!/bin/bash
# Round 6: kernel 1's LDS-resident runs with the top stack word kept in
# registers (ab/k1_top1.so: ab/k1_topreg.diff applied, built with -DMG_K1_TOPREG=1) against the shipped all-LDS form: kernel-1
# parity on the variant first, then interleaved processes on the bench's C2 batch.
# (profiles/r06/ab_k1top/ was measured with the roles swapped: TOPREG=1 was then the default.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-_top}
mkdir -p $OUT
MYTHGPU_LIB=$PWD/ab/k1_top1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread \
    tests/test_gpu_lanes.py tests/test_gpu_bench_fidelity.py tests/test_gpu_lds_plan.py \
    tests/test_gpu_lanes_per_wave.py tests/test_gpu_regrow.py tests/test_gpu_state_pins.py \
    > $OUT/parity_top.log 2>&1 && \
timeout -k 10 600 python -u scripts/ab_libs.py ab/k1_top1.so mythril_amd/libmythgpu.so 4 \
    > $OUT/ab_k1top.log 2>&1
