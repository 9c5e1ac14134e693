#!/usr/bin/env python3
"""Kernel-1 time of the C2 batch vs the per-launch step budget: fixed launch
cost and per-step slope of the real workload (cf. scripts/opbench.py)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mythril_amd import workloads  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.lanes import bucket_order, permuted  # noqa: E402


def main():
    dev = GpuDevice(0)
    cid = dev.load_code(workloads.bytecode("overflow.sol.o"))
    stop = dev.load_code(b"\x00")
    b = workloads.c2_batch(65536, code_id=cid, stack_cap=1024, mem_cap=1024, rec_cap=128)
    b = permuted(b, bucket_order(b))
    for cov in (False, True):
        run(dev, b, cov, [1, 2, 5, 10, 25, 50, 100, 150, 200, 1 << 30])
    b.code_id[:] = stop
    run(dev, b, True, [1 << 30])


def run(dev, b, cov, budgets):
    dev.alloc(b.shape, coverage=cov)
    dev.upload(workloads.slim_copy(b))
    print(f"coverage {cov}  code {int(b.code_id[0])}")
    for k in budgets:
        best = None
        for _ in range(3):
            dev.reset()
            st = dev.step(max_steps=k)
            best = st.kernel_ms if best is None else min(best, st.kernel_ms)
        print(f"max_steps {k:>10d}  kernel {best * 1000:8.1f} us  lane_steps {st.lane_steps:>9d}  "
              f"running {st.running}", flush=True)


if __name__ == "__main__":
    main()
