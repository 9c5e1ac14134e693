#!/usr/bin/env python3
"""A/B of library builds (compile-time variants) and lane orders on the bench's
C2 batch: each round runs one short process per variant (MYTHGPU_LIB, ORDER)
and takes its C2 kernel time; rounds alternate the order.
usage: ab_libs.py libA.so[:wave] libB.so[:wave] ... [rounds]
(`:wave` = lanes.wave_aligned_order instead of bucket_order)"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CHILD = r'''
import os, sys, json, numpy as np
sys.path.insert(0, os.environ["GRAFT_ROOT"])
from mythril_amd import workloads
from mythril_amd.device import GpuDevice
from mythril_amd.lanes import bucket_order, permuted, wave_aligned_order
dev = GpuDevice(0)
cid = dev.load_code(workloads.bytecode("overflow.sol.o"))
b = workloads.c2_batch(65536, code_id=cid, stack_cap=1024, mem_cap=1024, rec_cap=128)
b = permuted(b, wave_aligned_order(b, workloads.C2_SELECTORS) if os.environ.get("ORDER") == "wave"
             else bucket_order(b))
dev.alloc(b.shape, coverage=True)
dev.upload(workloads.slim_copy(b))
dev.run_batches(3)
ms = []
for _ in range(5):
    st = dev.run_batches(10)
    ms.append(sum(s.kernel_ms for s in st) / len(st))
steps = st[0].lane_steps
print(json.dumps({"min_ms": min(ms), "steps": steps}))
'''


def main():
    args = sys.argv[1:]
    rounds = int(args.pop()) if args and args[-1].isdigit() else 3
    libs = args
    res = {l: [] for l in libs}
    for r in range(rounds):
        for lib in (libs if r % 2 == 0 else libs[::-1]):
            path, _, order = lib.partition(":")
            env = dict(os.environ, MYTHGPU_LIB=str(Path(path).resolve()), GRAFT_ROOT=str(ROOT),
                       ORDER=order or "bucket")
            out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                                 timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            if not line:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            res[lib].append(json.loads(line[0]))
            print(lib, res[lib][-1], flush=True)
    for lib, rs in res.items():
        best = min(x["min_ms"] for x in rs)
        print(json.dumps({"lib": lib, "best_ms": best, "G_lane_steps_s": rs[0]["steps"] / best / 1e6,
                          "steps": rs[0]["steps"]}), flush=True)


if __name__ == "__main__":
    main()
