#!/usr/bin/env python3
"""A/B of kernel 2 variants on the bench's C4 batch (1M DAGs x 4096 models):
models per thread (MG_BV_MPT, read at upload) in one process, and optionally a
second library build in a child process (MYTHGPU_LIB).  Every variant's
(first_sat, sat_count) must equal the first variant's.
usage: ab_k2.py [rounds] [other_lib.so]"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def measure(dev, prog, models, reps=3):
    dev.eval_upload(prog, models)
    dev.eval_run()
    ms = min(dev.eval_run() for _ in range(reps))
    fs, sc = dev.eval_download()
    return ms, fs, sc


def main():
    import numpy as np
    from mythril_amd.device import GpuDevice
    from mythril_amd.smt import synth
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    other = sys.argv[2] if len(sys.argv) > 2 else None
    t = time.time()
    prog, models = synth.c4_batch(1_000_000, 4096)
    print(f"c4 batch built in {time.time() - t:.1f}s", flush=True)
    if os.environ.get("AB_K2_CHILD"):
        dev = GpuDevice(0)
        ms, fs, sc = measure(dev, prog, models)
        np.savez(os.environ["AB_K2_CHILD"], fs=fs, sc=sc)
        print(json.dumps({"ms": ms}), flush=True)
        return
    dev = GpuDevice(0)
    res, ref = {}, None
    for r in range(rounds):
        order = ["1", "2", "4"] if r % 2 == 0 else ["4", "2", "1"]
        for m in order:
            os.environ["MG_BV_MPT"] = m
            ms, fs, sc = measure(dev, prog, models)
            if ref is None:
                ref = (fs, sc)
            assert np.array_equal(fs, ref[0]) and np.array_equal(sc, ref[1]), f"MPT={m} differs"
            res.setdefault(f"mpt{m}", []).append(ms)
            print(f"round {r} mpt {m}: {ms:.2f} ms", flush=True)
    os.environ.pop("MG_BV_MPT", None)
    dev.close()
    if other:
        out = "/tmp/ab_k2_child.npz"
        for r in range(max(1, rounds // 2)):
            env = dict(os.environ, MYTHGPU_LIB=str(Path(other).resolve()), AB_K2_CHILD=out)
            p = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=600)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if not line:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            d = np.load(out)
            assert np.array_equal(d["fs"], ref[0]) and np.array_equal(d["sc"], ref[1]), "other lib differs"
            res.setdefault("other", []).append(json.loads(line[0])["ms"])
            print(f"other lib: {res['other'][-1]:.2f} ms", flush=True)
    evals = prog.n_dags * models.n_models
    for k, v in res.items():
        print(json.dumps({"variant": k, "best_ms": min(v), "G_evals_s": evals / min(v) / 1e6}), flush=True)


if __name__ == "__main__":
    main()
