"""Which instructions the symbolic co-simulation's lanes escape to the host,
per contract: tests/symcases.run_both on the GPU."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import pytest  # noqa: E402

import symcases  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402

dev = GpuDevice(0)
out = {}
for name in symcases.ALL_CASES:
    mp = pytest.MonkeyPatch()
    try:
        got, want, laser = symcases.run_both(dev, name, mp)
        out[name] = {"equal": got == want, "escaped": dict(laser.escaped_ops), "lane_steps": int(laser.lane_steps)}
    finally:
        mp.undo()
    print(name, json.dumps(out[name]), flush=True)
for name in symcases.SYM_CREATIONS_ALL:
    mp = pytest.MonkeyPatch()
    try:
        got, want, laser = symcases.run_creation_both(dev, name, mp)
        out["creation:" + name] = {"equal": got == want, "escaped": dict(laser.escaped_ops),
                                   "lane_steps": int(laser.lane_steps)}
    finally:
        mp.undo()
    print("creation:" + name, json.dumps(out["creation:" + name]), flush=True)
dev.close()
