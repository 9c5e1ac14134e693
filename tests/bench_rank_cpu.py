"""One rank of bench.py on the CPU (gloo + the oracle stand-in device): the
script tests/test_bench_launcher.py hands to bench.launch_ranks, so the rank
launcher, the weak-scaling reduction and the coverage all-gather run exactly as
on the GPU box, with oracle/evm_ref.c in place of kernel 1.  Test infrastructure."""
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE))

import bench  # noqa: E402
from oracle_device import OracleDevice  # noqa: E402

if __name__ == "__main__":
    bench.main(sys.argv[1:], device_factory=lambda local: OracleDevice(), backend="gloo")
