#!/bin/bash
# Instruction-cache counters of kernel 1 on the C2 bench (one rocprofv3 pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_BUSY_CYCLES SQ_IFETCH SQ_WAVES SQ_BUSY_CYCLES -d $OUT/pmc_ic -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $OUT/pmc_ic.log 2>&1
