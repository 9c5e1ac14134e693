#!/bin/bash
# SQ counter passes (one group per rocprofv3 run) over a short bench: VALU
# utilisation, instruction mix, LDS bank conflicts and wait states of both kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-dags 131072 --c4-steps 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc_sq1 -o run --output-format csv -- $B > $OUT/pmc_sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH -d $OUT/pmc_sq2 -o run --output-format csv -- $B > $OUT/pmc_sq2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_ACCUM_PREV_HIRES -d $OUT/pmc_sq3 -o run --output-format csv -- $B > $OUT/pmc_sq3.log 2>&1
echo done
