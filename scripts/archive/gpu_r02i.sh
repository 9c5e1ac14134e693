#!/bin/bash
# Round-2 profiles: laser/bench-fidelity tests, bench line, kernel trace,
# HBM passes, SQ passes on the bench and on the kernel-2 op classes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02i
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 1 --unbucketed-steps 0 --profile-only"
echo "== tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu_laser.py tests/test_gpu_bench_fidelity.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 && \
echo "== bench" && timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && \
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --unbucketed-steps 0 --profile-only > $OUT/prof_trace.log 2>&1 && \
echo "== fetch" && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- $B > $OUT/prof_fetch.log 2>&1 && \
echo "== write" && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- $B > $OUT/prof_write.log 2>&1 && \
echo "== sq_a" && timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc_sq_a -o run --output-format csv -- $B > $OUT/pmc_sq_a.log 2>&1 && \
echo "== sq_b" && timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY -d $OUT/pmc_sq_b -o run --output-format csv -- $B > $OUT/pmc_sq_b.log 2>&1 && \
echo "== k2 classes" && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc_k2cls -o run --output-format csv -- python3 scripts/k2_opclass.py > $OUT/k2_opclass.log 2>&1 && \
echo "== done"
