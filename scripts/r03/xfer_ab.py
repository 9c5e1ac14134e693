"""A/B of the lane transfers (mg_lanes_upload / mg_lanes_download_live) as
LaserEVM issues them: the batched plan (one pinned DMA + one sync per phase)
against MG_XFER=legacy (one pageable copy + sync per field).  A C2 batch of
4,096 lanes (LaserEVM's hooked_c2 shape: stack_cap 64, mem_cap 1024, rec_cap
128) is stepped once so lanes hold real stacks / memory, then ranges of 1, 64
and 4,096 lanes are downloaded live and uploaded back, 50 times each; the
downloaded image must be identical under both paths."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from mythril_amd import workloads  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402


def run(mode):
    if mode == "legacy":
        os.environ["MG_XFER"] = "legacy"
    else:
        os.environ.pop("MG_XFER", None)
    dev = GpuDevice(0)
    b = workloads.c2_batch(4096, stack_cap=64, mem_cap=1024, rec_cap=128)
    b.code_id[:] = dev.load_code(workloads.bytecode("overflow.sol.o"))
    dev.alloc(b.shape)
    dev.upload(b)
    dev.step(max_steps=40)
    out = {}
    images = {}
    for n in (1, 64, 4096):
        dev.download_range(b, 0, n, live=True)
        t0 = time.perf_counter()
        for _ in range(50):
            dev.download_range(b, 0, n, live=True)
        t1 = time.perf_counter()
        for _ in range(50):
            dev.upload_range(b, 0, n)
        t2 = time.perf_counter()
        for _ in range(50):
            dev.upload_range(b, 0, n, live=True)
        t3 = time.perf_counter()
        out[n] = {"download_ms": (t1 - t0) / 50 * 1e3, "upload_ms": (t2 - t1) / 50 * 1e3,
                  "upload_live_ms": (t3 - t2) / 50 * 1e3}
    dev.download(b)
    images = {k: np.array(getattr(b, k)).copy() for k in ("pc", "sp", "msize", "steps", "stack", "memory",
                                                          "storage", "gas_min", "rec_len", "rec")}
    dev.close()
    return out, images


if __name__ == "__main__":
    res = {}
    imgs = {}
    for mode in ("batched", "legacy", "batched"):
        r, im = run(mode)
        res.setdefault(mode, []).append(r)
        imgs.setdefault(mode, im)
    same = all(np.array_equal(imgs["batched"][k], imgs["legacy"][k]) for k in imgs["batched"])
    print(json.dumps({"same_image": same, "results": res}, indent=1))
    if not same:
        sys.exit(1)
