#!/usr/bin/env python3
"""Round 5: C2 at 64 and 32 lanes per wave (MG_LANES_PER_WAVE, read by mg_open:
one child process per variant), interleaved rounds, on the bench's C2 batch --
the measurement that prices a limb split: 32 paths per wave
is 2 waves per SIMD with the instruction stream unchanged.  Every variant's
lane results (steps and statuses) must be the first's."""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def child():
    import numpy as np
    from mythril_amd import workloads
    from mythril_amd.device import GpuDevice
    from mythril_amd.lanes import LaneBatch, bucket_order, permuted
    dev = GpuDevice(0)
    code = workloads.bytecode("overflow.sol.o")
    cid = dev.load_code(code)
    batch = workloads.c2_batch(65536, code_id=cid, seed=workloads.C2_SEED, stack_cap=1024, mem_cap=1024,
                               rec_cap=128)
    batch = permuted(batch, bucket_order(batch))
    dev.alloc(batch.shape, coverage=True)
    dev.upload(workloads.slim_copy(batch))
    dev.run_batches(3)
    t = time.perf_counter()
    st = dev.run_batches(20)
    wall = time.perf_counter() - t
    out = LaneBatch(batch.shape)
    dev.download(out)
    steps = sum(s.lane_steps for s in st)
    print(json.dumps({"kernel_ms": float(np.mean([s.kernel_ms for s in st])), "G": steps / wall / 1e9,
                      "check": [int(out.steps.sum()), int(out.status.astype(np.int64).sum())]}), flush=True)
    dev.close()


def main(rounds=3):
    res, ref = {}, None
    for r in range(rounds):
        for lpw in ((64, 32) if r % 2 == 0 else (32, 64)):
            env = dict(os.environ, MG_LANES_PER_WAVE=str(lpw), AB_LPW_CHILD="1")
            p = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode or not line:
                print(p.stdout[-2000:], p.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            d = json.loads(line[0])
            ref = ref or d["check"]
            assert d["check"] == ref, (lpw, d["check"], ref)
            res.setdefault(lpw, []).append(d)
            print(f"round {r} lanes/wave {lpw}: {d['kernel_ms']:.4f} ms/launch, {d['G']:.2f} G lane-steps/s", flush=True)
    for lpw, ds in res.items():
        print(json.dumps({"lanes_per_wave": lpw, "best_kernel_ms": min(x["kernel_ms"] for x in ds),
                          "best_G": max(x["G"] for x in ds)}), flush=True)


if __name__ == "__main__":
    child() if os.environ.get("AB_LPW_CHILD") else main()
