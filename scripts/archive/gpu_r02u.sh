#!/bin/bash
# Kernel 2 at 8 waves per SIMD with scalar-load fetch: its parity tests, the full GPU
# suite, smoke, the bench line, the kernel trace and the HBM passes of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02u
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 1 --unbucketed-steps 0 --profile-only"
echo "== k2" && timeout -k 10 600 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_solver.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_k2.log 2>&1 && \
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
echo "== bench" && timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --unbucketed-steps 0 --profile-only > $OUT/prof_trace.log 2>&1 && \
echo "== fetch" && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- $B > $OUT/prof_fetch.log 2>&1 && \
echo "== write" && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- $B > $OUT/prof_write.log 2>&1 && \
echo "== done"
