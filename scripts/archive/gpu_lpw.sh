#!/bin/bash
# Kernel-1 lanes-per-wave A/B: kernel-1 parity tests at 32 and 16 lanes per wave,
# then C2 bench lines at 64, 32 and 16 (MG_LANES_PER_WAVE).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for L in 32 16; do
  MG_LANES_PER_WAVE=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_laser.py -x -q --timeout 300 --timeout-method thread > $OUT/lpw_pytest_$L.log 2>&1 || exit 1
done
for L in 64 32 16 64 32 16; do
  MG_LANES_PER_WAVE=$L timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-c4 >> $OUT/lpw_bench_$L.log 2>&1 || exit 1
done
echo done
