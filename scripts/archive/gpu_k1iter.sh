#!/bin/bash
# Kernel-1 iteration: parity tests, two C2 bench lines, SHA3 opbench and the clock bins.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_laser.py tests/test_gpu_creation.py -x -q --timeout 300 --timeout-method thread > $OUT/it_pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-c4 >> $OUT/it_bench.log 2>&1 || exit 1
done
timeout -k 10 300 python -u scripts/opbench.py 65536 ${PATTERNS:-sha3_64,push1_pop,mstore_mload} > $OUT/it_opbench.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/k1_clocks.py > $OUT/it_clocks.log 2>&1
