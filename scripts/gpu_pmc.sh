#!/bin/bash
# PMC passes on the C2 lane-step kernel (one counter group per rocprofv3 run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c4"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc_sq1 -o run --output-format csv -- $B > $OUT/pmc_sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT -d $OUT/pmc_sq2 -o run --output-format csv -- $B > $OUT/pmc_sq2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $OUT/pmc_sqc -o run --output-format csv -- $B > $OUT/pmc_sqc.log 2>&1
echo done
