#!/bin/bash
# Round 5: issue-rate probe, then the integration / taint / symbolic GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r05${1:-g}
mkdir -p $OUT
timeout -k 10 120 hipcc --offload-arch=gfx950 -O3 scripts/probes/issue_rates.hip -o /tmp/issue_rates > $OUT/probe_build.log 2>&1 && \
timeout -k 10 60 /tmp/issue_rates > $OUT/issue_rates.json 2> $OUT/issue_rates.err && \
timeout -k 10 880 python -u -m pytest tests/test_gpu_integration.py tests/test_gpu_taint.py tests/test_gpu_symbolic.py -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
