#!/bin/bash
# Round 5: SQ counters of kernel 2 on the bench's C4 launch (scripts/r03/k2_c4.py), the input of
# the issue floor the bench line reports (mythril_amd/roofline.k2_issue_floor).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-o}
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $OUT/c4sq -o run --output-format csv -- python3 -u scripts/r03/k2_c4.py > $OUT/c4sq.log 2>&1
