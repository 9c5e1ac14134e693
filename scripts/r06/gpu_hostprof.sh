#!/bin/bash
# Round 6: host profiles (cProfile) of the in-situ fields on the MI355X, with the exact
# procedure behind kernel 2: symbolic_tx exceptions / overflow (2 replicas) and myth_analyze.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r06${1:-_hp}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/r05/prof_symtx.py $OUT/prof_symtx_exceptions.txt exceptions.sol.o 2 gpu \
    > $OUT/prof_symtx.log 2>&1 && \
timeout -k 10 300 python -u scripts/r05/prof_symtx.py $OUT/prof_symtx_overflow.txt overflow.sol.o 2 gpu \
    >> $OUT/prof_symtx.log 2>&1 && \
timeout -k 10 400 python -u scripts/r05/prof_analyze.py $OUT/prof_analyze.txt > $OUT/prof_analyze.log 2>&1
