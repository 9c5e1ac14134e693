#!/bin/bash
# Round 4: kernel traces of the symbolic / taint lane transfers (LDS-tiled transpose kernels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04${1:-o}
mkdir -p $OUT
for kind in symbolic taint; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sym_${kind}_trace -o run --output-format csv -- python3 -u scripts/r04/sym_timed.py $kind > $OUT/sym_${kind}_trace.log 2>&1 || exit 1
done
