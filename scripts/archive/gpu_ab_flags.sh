#!/bin/bash
# A/B of compiler-flag variants of libmythgpu.so (ab/*.so): C2 + C4 bench line per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for v in base ${VARIANTS:-lib_o2 lib_nosink lib_nounroll}; do
  if [ $v = base ]; then L=$PWD/mythril_amd/libmythgpu.so; else L=$PWD/ab/$v.so; fi
  echo "== $v"
  MYTHGPU_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --c4-steps 2 > $OUT/abf_$v.log 2>&1 || exit 1
done
