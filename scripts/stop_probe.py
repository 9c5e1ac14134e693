#!/usr/bin/env python3
"""Fixed cost of one kernel-1 launch: lanes whose code is a lone STOP, at
several batch sizes (prologue, staging, epilogue and dispatch, no stepping)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from mythril_amd import workloads  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.lanes import LaneBatch, LaneShape  # noqa: E402


def main():
    dev = GpuDevice(0)
    dev.load_code(workloads.bytecode("overflow.sol.o"))     # sizes the LDS plan like C2
    stop = dev.load_code(b"\x00")
    for n in [256, 4096, 16384, 65536]:
        for cov in (False, True):
            b = LaneBatch(LaneShape(n=n, stack_cap=1024, mem_cap=1024, calldata_cap=96, storage_cap=16))
            for i in range(n):
                b.set_lane(i, code_id=stop)
            dev.alloc(b.shape, coverage=cov)
            dev.upload(b)
            best = 1e9
            for _ in range(5):
                dev.reset()
                best = min(best, dev.step().kernel_ms)
            print(f"lanes {n:6d} coverage {cov!s:5s} kernel {best * 1000:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
