#!/bin/bash
# Round 5: k_lane_step's SQ counters on the C2 launches of the bench's profile command (two
# passes of at most 8 SQ counters), for the line's issue_floor / counter_fracs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-k1sq}
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --unbucketed-steps 0 --profile-only"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/k1_sq_a -o run --output-format csv -- $B > $OUT/k1_sq_a.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $OUT/k1_sq_b -o run --output-format csv -- $B > $OUT/k1_sq_b.log 2>&1
