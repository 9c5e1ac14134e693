#!/usr/bin/env python3
"""Distinct paths per wave of the bench's C2 batch (CPU oracle): lanes stepped
one instruction at a time, each lane's path = its pc sequence; a wave of 64
consecutive lanes (bucketed order) pays for the union of its lanes' paths."""
import collections
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

from mythril_amd import workloads  # noqa: E402
from mythril_amd.lanes import MG_RUNNING, bucket_order, permuted  # noqa: E402
from oracle.evm_ref import OracleEVM  # noqa: E402


def paths(b, code):
    o = OracleEVM()
    cid = o.load_code(code)
    b = b.copy()
    b.code_id[:] = cid
    n = b.n
    h = np.zeros(n, dtype=np.uint64)
    for _ in range(2000):
        live = b.status == MG_RUNNING
        if not live.any():
            break
        h[live] = h[live] * np.uint64(1000003) + b.pc[live].astype(np.uint64) + np.uint64(1)
        o.run(b, max_steps=1)
    return h, b.steps.copy()


def main(n=65536, code_name="overflow.sol.o"):
    code = workloads.bytecode(code_name) if code_name != "large" else workloads.large_code()
    kw = {} if code_name != "large" else {"selectors": workloads.dispatch_selectors(code)}
    b = workloads.c2_batch(n, stack_cap=64, mem_cap=4096, **kw)
    b = permuted(b, bucket_order(b))
    h, steps = paths(b, code)
    W = 64
    nd = [len(set(h[w:w + W].tolist())) for w in range(0, n, W)]
    cost = [sum(int(steps[w:w + W][h[w:w + W] == p][0]) for p in set(h[w:w + W].tolist()))
            for w in range(0, n, W)]
    print("distinct paths in batch:", len(set(h.tolist())))
    print("waves by distinct paths:", sorted(collections.Counter(nd).items()))
    c = np.array(cost)
    print(f"serial steps per wave: mean {c.mean():.0f} p50 {np.median(c):.0f} p90 {np.percentile(c, 90):.0f} "
          f"max {c.max()}  (lane steps mean {steps.mean():.0f} max {steps.max()})")
    top = collections.Counter(h.tolist()).most_common(12)
    print("largest path groups (lanes, steps):",
          [(k, int(steps[h == p][0])) for p, k in top])


if __name__ == "__main__":
    main(*(int(a) if a.isdigit() else a for a in sys.argv[1:]))
