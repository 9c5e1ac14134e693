#!/bin/bash
# north_star's rocprof evidence for both kernels: LDS bank conflicts and VALU
# thread utilisation (divergence), one counter pass per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02x
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 1 --unbucketed-steps 0 --profile-only"
echo "== list" && timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 ; \
echo "== lds" && timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL -d $OUT/pmc_lds -o run --output-format csv -- $B > $OUT/pmc_lds.log 2>&1 && \
echo "== valu" && timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d $OUT/pmc_valu -o run --output-format csv -- $B > $OUT/pmc_valu.log 2>&1 && \
echo "== done"
