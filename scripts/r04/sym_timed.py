#!/usr/bin/env python3
"""k_sym_step's timed launches alone, for PMC passes: the
symbolic_lanes field (no profiling pass) or the taint_lanes field, one kind per
process, so the counters describe exactly the launches the bench divides by."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402


def main(kind: str, order: str = "code"):
    dev = GpuDevice(0)
    if kind == "symbolic":
        out = bench.run_symbolic_lanes(dev, 65536, reps=5, profile=False, order=order)
    else:
        out = bench.run_taint_lanes(dev, 65536, reps=5, order=order, profile=False)
    print(json.dumps({kind: out}), flush=True)
    dev.close()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "symbolic", sys.argv[2] if len(sys.argv) > 2 else "code")
