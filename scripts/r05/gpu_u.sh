#!/bin/bash
# Round 5: the whole -m gpu suite on the build with k_sym_step's argument structs out of scratch
# and kernel 2's combined epilogue test; k_sym_step's PMC passes; kernel 2's C4 SQ pass; host
# profiles of symbolic_tx; the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-u}
OUT=gpurun_out/r05$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
AB_K2_MODES=scalar timeout -k 10 700 python3 -u scripts/ab_k2.py 3 ab/k2_v14.so > $OUT/ab_k2.log 2>&1 && \
bash scripts/r05/gpu_sympmc.sh $T code && \
bash scripts/r05/gpu_k2c4sq.sh $T && \
timeout -k 10 300 python -u scripts/r05/prof_symtx.py $OUT/hostprof_exceptions.txt exceptions.sol.o 8 gpu > $OUT/hostprof.log 2>&1 && \
timeout -k 10 300 python -u scripts/r05/prof_symtx.py $OUT/hostprof_overflow.txt overflow.sol.o 8 gpu >> $OUT/hostprof.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
