#!/bin/bash
# Round 5: kernel 2's per-op-class SQ pass (scripts/k2_opclass.py: C4 mix + one launch set per
# class) -- instruction counts by class per wave, for the issue-bound floor.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-q}
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/k2sq -o run --output-format csv -- python3 -u scripts/k2_opclass.py > $OUT/k2sq.log 2>&1
