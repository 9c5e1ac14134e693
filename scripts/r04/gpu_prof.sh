#!/bin/bash
# Round 4 evidence: symbolic_tx host cProfile; kernel-2 SQ passes on the shipped
# (fused, trimmed) build; k_sym_step FETCH/WRITE on the timed launches alone
# (symbolic and taint separately); kernel-1 per-wave clock bins on this tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-c}
mkdir -p $OUT/hostprof
K="python3 -u scripts/r03/k2_c4.py"
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c4 --hooked-lanes 0 --overlap-steps 0 \
    --unbucketed-steps 0 --large-steps 0 --taint-lanes 0 --symbolic-lanes 0 --host-profile $OUT/hostprof \
    > $OUT/bench_symtx.json 2> $OUT/bench_symtx.err && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/k2_sq_a -o run --output-format csv -- $K > $OUT/k2_sq_a.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $OUT/k2_sq_b -o run --output-format csv -- $K > $OUT/k2_sq_b.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/k2_fetch -o run --output-format csv -- $K > $OUT/k2_fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/k2_write -o run --output-format csv -- $K > $OUT/k2_write.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k2_trace -o run --output-format csv -- $K > $OUT/k2_trace.log 2>&1 && \
for kind in symbolic taint; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sym_${kind}_trace -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py $kind > $OUT/sym_${kind}_trace.log 2>&1 && \
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/sym_${kind}_fetch -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py $kind > $OUT/sym_${kind}_fetch.log 2>&1 && \
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/sym_${kind}_write -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py $kind > $OUT/sym_${kind}_write.log 2>&1 || exit 1
done && \
timeout -k 10 300 python3 -u scripts/k1_clocks.py > $OUT/k1_clocks.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/k1_sq_a -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --unbucketed-steps 0 --profile-only > $OUT/k1_sq_a.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $OUT/k1_sq_b -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --unbucketed-steps 0 --profile-only > $OUT/k1_sq_b.log 2>&1
