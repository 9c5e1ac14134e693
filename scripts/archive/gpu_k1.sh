#!/bin/bash
# Kernel-1 iteration: lane parity tests, C2 bench, per-opcode microbenchmark.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_laser.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_k1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4 > $OUT/bench_k1.log 2>&1 && \
timeout -k 10 300 python -u scripts/opbench.py 65536 push1_pop,add,jumpdest,mstore_mload,sload > $OUT/opbench.log 2>&1
