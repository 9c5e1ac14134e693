#!/bin/bash
# Round 3 evidence: the C2 kernel trace of the bench's timed path (--profile-only),
# and k_sym_step's trace, HBM passes and SQ passes at 65,536 symbolic / taint lanes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-s}
mkdir -p $OUT
S="python3 -u scripts/r03/sym_lanes.py"
K="python3 -u scripts/r03/k2_c4.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --unbucketed-steps 0 --profile-only > $OUT/prof_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/sym_trace -o run --output-format csv -- $S > $OUT/sym_trace.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- $S > $OUT/sym_fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- $S > $OUT/sym_write.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc_sq_a -o run --output-format csv -- $S > $OUT/sym_sq_a.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $OUT/pmc_sq_b -o run --output-format csv -- $S > $OUT/sym_sq_b.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/k2_fetch -o run --output-format csv -- $K > $OUT/k2_fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/k2_write -o run --output-format csv -- $K > $OUT/k2_write.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/k2_sq_a -o run --output-format csv -- $K > $OUT/k2_sq_a.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $OUT/k2_sq_b -o run --output-format csv -- $K > $OUT/k2_sq_b.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/k2_cls -o run --output-format csv -- python3 -u scripts/k2_opclass.py > $OUT/k2_cls.log 2>&1
