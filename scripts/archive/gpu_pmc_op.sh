#!/bin/bash
# SQ instruction counters of kernel 1 per opcode pattern (scripts/opbench.py), one
# rocprofv3 pass per pattern.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for p in ${PATTERNS:-push1_pop jumpdest jumpi_fall caller_pop add}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY -d $OUT/pmcop_$p -o run --output-format csv -- python3 scripts/opbench.py 65536 $p > $OUT/pmcop_$p.log 2>&1 || exit 1
done
