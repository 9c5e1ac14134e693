#!/bin/bash
# Round-2 final evidence on the final tree: the GPU suite, smoke, kernel-2 op-class
# SQ pass (division VALU cost at 8 waves), the full bench line, the kernel trace
# and the HBM passes of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r02y
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --c4-steps 1 --unbucketed-steps 0 --profile-only"
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
echo "== smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
echo "== k2 classes" && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc_k2cls -o run --output-format csv -- python3 scripts/k2_opclass.py > $OUT/k2_opclass.log 2>&1 && \
echo "== div valu" && python3 scripts/k2_div_valu.py $OUT/pmc_k2cls/run_counter_collection.csv $OUT/k2_opclass.log $OUT/k2_div_valu.json > $OUT/k2_div_valu.log 2>&1 && \
cp $OUT/k2_div_valu.json profiles/r02/k2_div_valu.json && \
echo "== bench" && timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && \
echo "== trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --unbucketed-steps 0 --profile-only > $OUT/prof_trace.log 2>&1 && \
echo "== fetch" && timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run --output-format csv -- $B > $OUT/prof_fetch.log 2>&1 && \
echo "== write" && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run --output-format csv -- $B > $OUT/prof_write.log 2>&1 && \
echo "== done"
