#!/bin/bash
# Round 3: kernel 2 DAG-major loop order -- creation test alone, kernel-2 parity,
# A/B against the chunk-major build (ab/k2_base.so), then the suite, smoke, bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbolic.py -k creation -v --timeout 240 --timeout-method thread > $OUT/pytest_creation.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "creation test rc=$rc: stop"; exit $rc; fi
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_eval.py tests/test_gpu_k2_pinning.py tests/test_gpu_solver.py > $OUT/pytest_k2.log 2>&1 || exit $?
timeout -k 10 600 python -u scripts/ab_k2.py 2 ab/k2_base.so > $OUT/ab_k2.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    --deselect "tests/test_gpu_symbolic.py::test_symbolic_creation_on_kernel1_equals_the_restatement[flag_array.sol.o]" \
    > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
