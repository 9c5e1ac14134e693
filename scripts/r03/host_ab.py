"""Within-one-box A/B of the host-path changes on bench.py's hooked_c2 field
(4,096 C2 lanes through LaserEVM with a counting hook on every opcode the
default modules hook): every variant in the same process, two interleaved
rounds, lane-steps/s each.
  all        the shipped path
  no_freeze  LaserEVM.exec without gc.freeze
  no_fast    the general MG_HOOK branch instead of _deliver_plain_hook
  legacy     + MG_XFER=legacy lane transfers (one pageable copy + sync per field)
The event counts must be equal in every variant."""
import gc
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import bench  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.laser import svm  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    devs = {"batched": GpuDevice(0)}
    os.environ["MG_XFER"] = "legacy"
    devs["legacy"] = GpuDevice(0)
    os.environ.pop("MG_XFER")
    real_freeze = gc.freeze
    variants = [("all", "batched", True, True), ("no_freeze", "batched", False, True),
                ("no_fast", "batched", True, False), ("legacy", "legacy", False, False)]
    res, events = {}, {}
    bench.run_hooked_c2(devs["batched"], 512, 0)          # warm-up (imports, code upload)
    for rnd in range(2):
        for name, dev, freeze, fast in (variants if rnd == 0 else variants[::-1]):
            gc.freeze = real_freeze if freeze else (lambda: None)
            svm.LaserEVM._fast_hooks = fast
            gc.collect()
            out = bench.run_hooked_c2(devs[dev], n, 0)
            res.setdefault(name, []).append(out["lane_steps_per_s"])
            events.setdefault(name, set()).add((out["lane_steps"], out["hook_events"], out["launches"]))
            print(name, rnd, round(out["lane_steps_per_s"]), round(out["wall_s"], 3), flush=True)
    gc.freeze = real_freeze
    svm.LaserEVM._fast_hooks = True
    assert len({e for v in events.values() for e in v}) == 1, events
    print(json.dumps({k: {"best_lane_steps_per_s": max(v), "runs": v} for k, v in res.items()}))


if __name__ == "__main__":
    main()
