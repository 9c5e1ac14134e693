#!/usr/bin/env python3
"""Two library contexts on one GPU after a one-batch warm-up only: the C2 batch
K times per context from two threads, against K times on one context.  The
first call with more batches than before allocates statistics slots and events;
measured on the MI355X (r02z) those first-use allocations serialise the two
streams (two contexts slower than one), which is why bench.run_two_streams
warms each context up at the timed batch count."""
import json
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(k=40):
    from mythril_amd import workloads
    from mythril_amd.device import GpuDevice
    from mythril_amd.lanes import bucket_order, permuted
    devs = [GpuDevice(0), GpuDevice(0)]
    for d in devs:
        cid = d.load_code(workloads.bytecode("overflow.sol.o"))
        b = workloads.c2_batch(65536, code_id=cid, stack_cap=1024, mem_cap=1024, rec_cap=128)
        b = permuted(b, bucket_order(b))
        d.alloc(b.shape, coverage=True)
        d.upload(workloads.slim_copy(b))
        d.run_batches(1)
    t = time.perf_counter()
    one = devs[0].run_batches(k)
    t1 = time.perf_counter() - t
    res = [None, None]

    def go(i):
        res[i] = devs[i].run_batches(k)
    t = time.perf_counter()
    th = [threading.Thread(target=go, args=(i,)) for i in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    t2 = time.perf_counter() - t
    s1 = sum(s.lane_steps for s in one)
    s2 = sum(s.lane_steps for r in res for s in r)
    print(json.dumps({"one_context_G": s1 / t1 / 1e9, "two_contexts_G": s2 / t2 / 1e9, "batches": k}))
    for d in devs:
        d.close()


if __name__ == "__main__":
    main()
