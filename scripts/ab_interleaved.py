#!/usr/bin/env python3
"""Same-process, interleaved A/B of runtime switches (read per launch/upload by
libmythgpu.so): kernel 2 MG_BV_MPT on C4 (1M DAGs x 4096 models, the bench
config) and kernel 1 MG_K1_RUNS on C2 (the bench batch).  Each round visits
every variant once, so clock drift and box-to-box variance hit all of them
alike.  Prints per-variant min / median over rounds."""
import json
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from mythril_amd import workloads  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.lanes import bucket_order, permuted  # noqa: E402
from mythril_amd.smt import synth  # noqa: E402


def k2(dev, variants, rounds, n_dags):
    prog, models = synth.c4_batch(n_dags, 4096)
    res = {v: [] for v in variants}
    ref = None
    for _ in range(rounds):
        for v in variants:
            os.environ["MG_BV_MPT"] = v
            dev.eval_upload(prog, models)
            dev.eval_run()
            res[v].append(min(dev.eval_run() for _ in range(2)))
            fs, sc = dev.eval_download()
            key = (int(sc.sum()), int(fs.astype("int64").sum()))
            assert ref is None or key == ref, (v, key, ref)
            ref = key
    for v, ms in res.items():
        print(json.dumps({"kernel": "k_bv_eval", "MG_BV_MPT": v, "min_ms": min(ms),
                          "median_ms": statistics.median(ms),
                          "G_evals_s": n_dags * 4096 / min(ms) / 1e6}), flush=True)


def k1(dev, variants, rounds, code_name="overflow.sol.o"):
    """variants: "VAR=value[,VAR2=value]" strings (env switches read per launch)."""
    code = workloads.bytecode(code_name) if code_name.endswith(".o") else workloads.large_code()
    cid = dev.load_code(code)
    sels = None if code_name.endswith(".o") else workloads.dispatch_selectors(code)
    kw = {} if sels is None else {"selectors": sels}
    b = workloads.c2_batch(65536, code_id=cid, stack_cap=1024, mem_cap=1024, rec_cap=128, **kw)
    b = permuted(b, bucket_order(b))
    dev.alloc(b.shape, coverage=True)
    dev.upload(workloads.slim_copy(b))
    res = {v: [] for v in variants}
    steps = None
    for _ in range(rounds):
        for v in variants:
            for kv in v.split(","):
                k, _, val = kv.partition("=")
                os.environ[k] = val
            dev.run_batches(2)
            st = dev.run_batches(10)
            res[v].append(sum(s.kernel_ms for s in st) / len(st))
            n = sum(s.lane_steps for s in st) // len(st)
            assert steps is None or n == steps, (v, n, steps)
            steps = n
            for kv in v.split(","):
                os.environ.pop(kv.partition("=")[0], None)
    for v, ms in res.items():
        print(json.dumps({"kernel": "k_lane_step", "code": code_name, "variant": v, "min_ms": min(ms),
                          "median_ms": statistics.median(ms),
                          "G_lane_steps_s": steps / min(ms) / 1e6}), flush=True)


def main():
    dev = GpuDevice(0)
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    if which == "k1":
        variants = sys.argv[2].split(";") if len(sys.argv) > 2 else ["MG_K1_RUNS=lds", "MG_K1_RUNS=reg"]
        code = sys.argv[3] if len(sys.argv) > 3 else "overflow.sol.o"
        rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
        k1(dev, variants, rounds, code)
    if which == "k2":
        k2v = sys.argv[2].split(",") if len(sys.argv) > 2 else ["1", "2", "4"]
        k2(dev, k2v, 4, 1_000_000)
    dev.close()


if __name__ == "__main__":
    main()
