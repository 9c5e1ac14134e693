#!/bin/bash
# Kernel 2 A/B (round 3): shared division site + masked-ops set + one-ahead
# scalar instruction fetch (in-tree, 8 waves) vs the round-2 build (ab/k2_old.so)
# vs the same sources at 7 waves (ab/k2_w7.so); then per-class timings and the
# SQ passes on the shipped build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-m}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_state_pins.py > $OUT/pytest_k2.log 2>&1 && \
timeout -k 10 600 python -u scripts/ab_k2.py 2 ab/k2_old.so ab/k2_w7.so > $OUT/ab_k2.log 2>&1 && \
timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmck2_a -o run --output-format csv -- python3 scripts/k2_opclass.py > $OUT/pmck2_a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $OUT/pmck2_b -o run --output-format csv -- python3 scripts/k2_opclass.py > $OUT/pmck2_b.log 2>&1 && \
timeout -k 10 300 python -u -c "
import json, sys
sys.path.insert(0, '.')
import bench
from mythril_amd.device import GpuDevice
dev = GpuDevice(0)
print(json.dumps(bench.run_symbolic_lanes(dev, 65536)))
" > $OUT/symlanes.json 2> $OUT/symlanes.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/symprof -o run -- python3 -u -c "
import json, sys
sys.path.insert(0, '.')
import bench
from mythril_amd.device import GpuDevice
dev = GpuDevice(0)
print(json.dumps(bench.run_symbolic_lanes(dev, 65536)))
" > $OUT/symprof.log 2>&1
