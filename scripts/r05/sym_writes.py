#!/usr/bin/env python3
"""Round 5 diagnostic: which lane planes one symbolic_lanes
launch of k_sym_step changes, in bytes per lane (upload, one launch, download,
compare plane by plane).  Bytes rewritten with the same value do not show."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.lanes import _ALL_FIELDS, _SYM_FIELDS, LaneBatch  # noqa: E402

dev = GpuDevice(0)
laser, b = bench.symbolic_lane_batch(dev, 65536)
dev.alloc(b.shape)
dev.upload(b)
st = dev.step()
out = LaneBatch(b.shape)
dev.download(out)
n = b.shape.n
res = {"lane_steps": int(st.lane_steps), "planes": {}}
for f in _ALL_FIELDS + _SYM_FIELDS:
    x, y = getattr(b, f, None), getattr(out, f, None)
    if x is None or y is None:
        continue
    xb = np.ascontiguousarray(x).view(np.uint8).reshape(n, -1)
    yb = np.ascontiguousarray(y).view(np.uint8).reshape(n, -1)
    diff = xb != yb
    changed = int(diff.sum())
    # 32-byte sectors touched per lane (dword-major planes are interleaved across lanes
    # on the device; this counts the lane's own changed bytes only)
    res["planes"][f] = {"bytes_per_lane": changed / n, "row_bytes": int(xb.shape[1])}
print(json.dumps(res, indent=1))
dev.close()
