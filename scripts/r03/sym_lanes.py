#!/usr/bin/env python3
"""k_sym_step at 65,536 lanes: bench.py's symbolic_lanes and taint_lanes fields
alone (the command the k_sym_step trace / PMC / SQ passes profile)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402


def main():
    dev = GpuDevice(0)
    out = {"symbolic_lanes": bench.run_symbolic_lanes(dev, 65536, reps=3),
           "taint_lanes": bench.run_taint_lanes(dev, 65536, reps=3)}
    print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
