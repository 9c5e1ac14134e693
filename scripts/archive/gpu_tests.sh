#!/bin/bash
# Full GPU parity suite + toolchain probe of the box (z3 / solc).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
(python -c "import z3; print('z3', z3.get_version_string())" 2>&1; which solc 2>&1; nproc; lscpu | grep "Model name") > $OUT/probe.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
