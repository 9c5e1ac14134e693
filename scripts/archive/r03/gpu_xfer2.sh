#!/bin/bash
# Round 3: the symbolic-creation test alone (its diff on failure), then the
# rest of the -m gpu suite, smoke and the default bench line.  A test failure
# (rc 1) does not stop the script; a fault, abort or time limit does.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_symbolic.py -k creation -v --timeout 240 --timeout-method thread > $OUT/pytest_creation.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "creation test rc=$rc: stop"; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    --deselect "tests/test_gpu_symbolic.py::test_symbolic_creation_on_kernel1_equals_the_restatement[flag_array.sol.o]" \
    > $OUT/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
