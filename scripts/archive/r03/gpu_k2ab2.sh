#!/bin/bash
# Kernel 2 A/B, second pass: the live-range-trimmed build (in-tree, 8 waves)
# against round 2 (ab/k2_old.so) and the same sources at 7 waves; per-launch
# HBM traffic (FETCH_SIZE, WRITE_SIZE passes) and the SQ passes of the shipped
# scalar-fetch build on the C4 batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-n}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py > $OUT/pytest_k2.log 2>&1 && \
timeout -k 10 600 python -u scripts/ab_k2.py 2 ab/k2_old.so ab/k2_w7b.so > $OUT/ab_k2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- python3 scripts/r03/k2_c4.py > $OUT/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- python3 scripts/r03/k2_c4.py > $OUT/pmc_write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc_sq_a -o run --output-format csv -- python3 scripts/r03/k2_c4.py > $OUT/pmc_sq_a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $OUT/pmc_sq_b -o run --output-format csv -- python3 scripts/r03/k2_c4.py > $OUT/pmc_sq_b.log 2>&1 && \
timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass.log 2>&1
