#!/bin/bash
# C2 after caching the LDS plan / switches per mg_run_batches call and copying the
# statistics through pinned memory: bench fidelity, the library A/B against
# round 2, and the bench's C2 line (--profile-only) three times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r03${1:-t}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_bench_fidelity.py tests/test_gpu_lds_plan.py > $OUT/pytest_c2.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_libs.py ab/k2_old.so mythril_amd/libmythgpu.so 4 > $OUT/ab_k1.log 2>&1 && \
for k in 1 2 3; do timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c4 --no-roofline --hooked-lanes 0 --taint-lanes 0 --symbolic-lanes 0 --symbolic-replicas 0 --unbucketed-steps 0 --overlap-steps 0 --large-steps 0 > $OUT/c2_$k.json 2> $OUT/c2_$k.err || exit 1; done
