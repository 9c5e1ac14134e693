#!/bin/bash
# Kernel-2 superinstructions (bv_fuse): parity (fused vs unfused vs oracle), C4
# A/B all shapes, two shapes and unfused in one library, op-class timings, then the GPU suite,
# smoke and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-f}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_eval.py \
    tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py > $OUT/pytest_k2.log 2>&1 && \
AB_K2_MODES=scalar,scalar-fuse4,scalar-fuse0 timeout -k 10 600 python -u scripts/ab_k2.py 2 > $OUT/ab_k2_fuse.log 2>&1 && \
timeout -k 10 300 python -u scripts/k2_opclass.py > $OUT/k2_opclass_fuse.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
# the bench's kernel trace and the HBM passes of its timed kernels (C2 + C4)
P="python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --unbucketed-steps 0 --profile-only"
if [ "${2:-}" = "prof" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --unbucketed-steps 0 --profile-only > $OUT/prof_trace.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/bench_pmc/prof_fetch -o run --output-format csv -- $P > $OUT/bench_fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/bench_pmc/prof_write -o run --output-format csv -- $P > $OUT/bench_write.log 2>&1
fi
