#!/bin/bash
# Round 5: kernel-2 A/B (in-tree vs variants), its SQ pass per op class on the in-tree build,
# the k_sym_step write experiment, and a host profile of the symbolic_tx field.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-m}
OUT=gpurun_out/r05$T
mkdir -p $OUT
AB_K2_MODES=scalar timeout -k 10 600 python3 -u scripts/ab_k2.py 3 ab/k2_base.so ab/k2_v5.so ab/k2_v6.so > $OUT/ab_k2.log 2>&1 && \
bash scripts/r05/gpu_k2sq.sh $T && \
bash scripts/r05/gpu_symflush.sh $T && \
timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 0 --no-c4 --no-cpu-baseline --hooked-lanes 0 --taint-lanes 0 --symbolic-lanes 0 --analyses 0 --overlap-steps 0 --unbucketed-steps 0 --large-steps 0 --no-roofline --host-profile $OUT/hostprof > $OUT/bench_symtx.log 2>&1
