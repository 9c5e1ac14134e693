#!/bin/bash
# Kernel-1 deferred-dispatch A/B: parity tests with the default defer set, then C2
# bench lines per MG_DEFER_KINDS mask (0 = off; 256 = SHA3; 196864 = SHA3, SLOAD,
# SSTORE; 221952 = those + CALLDATALOAD, MLOAD, MSTORE) and the clock bins.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_laser.py tests/test_gpu_creation.py tests/test_gpu_lanes_per_wave.py -x -q --timeout 300 --timeout-method thread > $OUT/defer_pytest.log 2>&1 || exit 1
for M in 0 256 196864 221952 0 256 196864 221952; do
  MG_DEFER_KINDS=$M timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-c4 >> $OUT/defer_bench_$M.log 2>&1 || exit 1
done
timeout -k 10 200 python -u scripts/k1_clocks.py > $OUT/defer_clocks.log 2>&1 || exit 1
MG_DEFER_KINDS=0 timeout -k 10 200 python -u scripts/k1_clocks.py > $OUT/defer_clocks_off.log 2>&1
