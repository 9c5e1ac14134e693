#!/bin/bash
# SQ counter passes on an opbench pattern (converged waves): per-iteration
# instruction mix and waits of kernel 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
PAT=${PAT:-jumpdest}
B="python3 scripts/opbench.py 65536 $PAT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/op_sq1 -o run --output-format csv -- $B > $OUT/op_sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM SQ_IFETCH -d $OUT/op_sq2 -o run --output-format csv -- $B > $OUT/op_sq2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES -d $OUT/op_sq3 -o run --output-format csv -- $B > $OUT/op_sq3.log 2>&1
echo done
