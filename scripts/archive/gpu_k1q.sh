#!/bin/bash
# Kernel-1 parity tests, SHA3 / EQ opbench patterns and two C2 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_laser.py tests/test_gpu_creation.py -x -q --timeout 300 --timeout-method thread > $OUT/k1q_pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/opbench.py 65536 ${PATTERNS:-sha3_64,eq_iszero,add} > $OUT/k1q_opbench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/k1q_bench1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/k1q_bench2.log 2>&1
