#!/bin/bash
# Round GPU check: parity tests, smoke, bench, rocprofv3 kernel trace + HBM counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
echo "== smoke" && timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
echo "== pytest" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== bench" && timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 8 > $OUT/bench.log 2>&1 && \
echo "== trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_trace.log 2>&1 && \
echo "== fetch" && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 1 > $OUT/prof_fetch.log 2>&1 && \
echo "== write" && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 1 > $OUT/prof_write.log 2>&1 && \
echo "== done"
