#!/bin/bash
# Kernel 2: op-class timing (LDS vs scalar program fetch) + SQ counter pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_lds.log 2>&1 && \
MG_BV_PROG=scalar timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_scalar.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmck2_c -o run --output-format csv -- python3 scripts/k2_opclass.py > $OUT/pmck2_c.log 2>&1
