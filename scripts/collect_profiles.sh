#!/bin/bash
# Copy the judged summaries of a scripts/archive/gpu_check.sh run from gpurun_out/ into profiles/<round>/.
set -e
R=${1:-r01}
D=profiles/$R
mkdir -p $D
cp gpurun_out/prof_trace/run_kernel_stats.csv $D/kernel_stats_trace.csv
cp gpurun_out/prof_fetch/run_counter_collection.csv $D/pmc_fetch_size.csv
cp gpurun_out/prof_write/run_counter_collection.csv $D/pmc_write_size.csv
cp gpurun_out/pytest_gpu.log $D/pytest_gpu.log
grep '^{' gpurun_out/bench.log | tail -1 > $D/bench.json
cp scripts/archive/gpu_check.sh $D/commands.sh
python3 scripts/pmc_summary.py gpurun_out $D
