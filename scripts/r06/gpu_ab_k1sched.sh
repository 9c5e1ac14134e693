#!/bin/bash
# Round 6: kernel-1 scheduler A/B -- the shipped build against the same
# sources compiled with -amdgpu-sched-strategy=gcn-max-ilp and -amdgpu-schedule-metric-bias=0,
# interleaved processes on the bench's C2 batch; then C2 parity of both variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-_k1}
mkdir -p $OUT
timeout -k 10 600 python -u scripts/ab_libs.py mythril_amd/libmythgpu.so ab/k1_ilp.so ab/k1_bias0.so 4 \
    > $OUT/ab_k1sched.log 2>&1 && \
MYTHGPU_LIB=$PWD/ab/k1_ilp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_bench_fidelity.py > $OUT/parity_ilp.log 2>&1 && \
MYTHGPU_LIB=$PWD/ab/k1_bias0.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_bench_fidelity.py > $OUT/parity_bias0.log 2>&1
