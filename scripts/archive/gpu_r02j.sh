#!/bin/bash
# LDS plan (staged prefix, memory window): parity tests, then interleaved A/Bs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02j
mkdir -p $OUT
echo "== lds tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu_lds_plan.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_lds.log 2>&1 && \
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== ab memwin" && timeout -k 10 300 python -u scripts/ab_interleaved.py k1 "MG_K1_MEMWIN=0;MG_K1_MEMWIN=128;MG_K1_MEMWIN=160;MG_K1_MEMWIN=192" > $OUT/ab_memwin.log 2>&1 && \
echo "== ab push" && timeout -k 10 300 python -u scripts/ab_interleaved.py k1 "MG_K1_PUSH=lds;MG_K1_PUSH=global" > $OUT/ab_push.log 2>&1 && \
echo "== ab large" && timeout -k 10 300 python -u scripts/ab_interleaved.py k1 "MG_K1_MEMWIN=0;MG_K1_MEMWIN=160;MG_K1_PD_CAP=1500" large 3 > $OUT/ab_large.log 2>&1 && \
echo "== done"
