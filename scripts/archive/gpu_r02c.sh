#!/bin/bash
# Kernel-2 A/B with SQ counters: r01 kernel (ab/lib_k2r01.so) vs the models-per-
# thread kernel at M=1 and M=2, C4 op mix (scripts/k2_c4mix.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02c
mkdir -p $OUT
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
PB="SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_VALU"
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u scripts/k2_c4mix.py > $OUT/$name.time 2>&1 || return 1
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $PA -d $OUT/$name.pa -o pmc -- python3 scripts/k2_c4mix.py > $OUT/$name.pa.log 2>&1 || return 1
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $PB -d $OUT/$name.pb -o pmc -- python3 scripts/k2_c4mix.py > $OUT/$name.pb.log 2>&1 || return 1
}
run r01 MYTHGPU_LIB=$PWD/ab/lib_k2r01.so &&
run m1 MG_BV_MPT=1 &&
run m2 MG_BV_MPT=2 &&
echo done
