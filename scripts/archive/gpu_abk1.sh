#!/bin/bash
# Kernel-1 A/B: C2 bench of ab/base.so vs ab/v1.so (interleaved), the lane/laser
# parity tests on v1, and an opcode microbenchmark subset on both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c4"
MYTHGPU_LIB=ab/v1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_laser.py -x -q --timeout 300 --timeout-method thread > $OUT/ab_pytest_v1.log 2>&1 || exit 1
for i in 1 2; do
  MYTHGPU_LIB=ab/base.so timeout -k 10 300 $B > $OUT/ab_base_$i.log 2>&1 && \
  MYTHGPU_LIB=ab/v1.so timeout -k 10 300 $B > $OUT/ab_v1_$i.log 2>&1 || exit 1
done
OPS=${OPS:-push1_pop,add,jumpdest,jumpi_fall,caller_pop,mstore_mload}
MYTHGPU_LIB=ab/base.so timeout -k 10 300 python -u scripts/opbench.py 65536 $OPS > $OUT/ab_op_base.log 2>&1 && \
MYTHGPU_LIB=ab/v1.so timeout -k 10 300 python -u scripts/opbench.py 65536 $OPS > $OUT/ab_op_v1.log 2>&1
