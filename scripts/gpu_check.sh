set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
python -c "import torch;print(torch.cuda.get_device_name(0))" > gpurun_out/dev.log 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 6 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
