#!/usr/bin/env python3
"""A/B of kernel 2 variants on the bench's C4 batch (1M DAGs x 4096 models):
the instruction fetch (MG_BV_PROG=lds|scalar, read at upload) for the in-tree
library and for every other library build given, each in a child process
(MYTHGPU_LIB).  Every variant's (first_sat, sat_count) must equal the first's.
usage: ab_k2.py [rounds] [other_lib.so[:legacy] ...] (legacy: C4 with concat(S0, acc),
for builds before the accumulator-in-A rule)"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def child():
    import numpy as np
    from mythril_amd.device import GpuDevice
    from mythril_amd.smt import synth
    prog, models = synth.c4_batch(1_000_000, 4096)
    dev = GpuDevice(0)
    out = {}
    for mode in os.environ.get("AB_K2_MODES", "lds,scalar").split(","):
        # "<fetch>-fuse<k>": the same fetch with MG_BV_FUSE=k (0: programs uploaded
        # unfused, 1: no binary-op shape, 2: pairs only, 3: no tails, 4: wide tails only,
        # 5: all, the default)
        fetch, _, fuse = mode.partition("-fuse")
        os.environ["MG_BV_PROG"] = fetch
        os.environ["MG_BV_FUSE"] = fuse or "5"
        dev.eval_upload(prog, models)
        dev.eval_run()
        ms = min(dev.eval_run() for _ in range(3))
        fs, sc = dev.eval_download()
        np.savez(f"{os.environ['AB_K2_CHILD']}.{mode}.npz", fs=fs, sc=sc)
        out[mode] = ms
    dev.close()
    print(json.dumps(out), flush=True)


def main():
    import numpy as np
    if os.environ.get("AB_K2_CHILD"):
        return child()
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    libs = [None] + sys.argv[2:]
    evals = 1_000_000 * 4096
    res, ref = {}, None
    for r in range(rounds):
        for lib in (libs if r % 2 == 0 else libs[::-1]):
            path, _, tag = (lib or "").partition(":")
            name = Path(path).stem if lib else "in-tree"
            out = f"/tmp/ab_k2_{name}"
            env = dict(os.environ, AB_K2_CHILD=out)
            if lib:
                env["MYTHGPU_LIB"] = str(Path(path).resolve())
            if tag == "legacy":           # a build before rconcat: C4's concat in the old form
                env["MYTH_C4_LEGACY_CONCAT"] = "1"
            t = time.time()
            p = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=900)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode or not line:
                print(p.stdout[-2000:], p.stderr[-3000:], file=sys.stderr)
                sys.exit(1)
            for mode, ms in json.loads(line[0]).items():
                d = np.load(f"{out}.{mode}.npz")
                if ref is None:
                    ref = (d["fs"], d["sc"])
                assert np.array_equal(d["fs"], ref[0]) and np.array_equal(d["sc"], ref[1]), f"{name}/{mode} differs"
                res.setdefault(f"{name}/{mode}", []).append(ms)
                print(f"round {r} {name}/{mode}: {ms:.2f} ms ({time.time() - t:.0f}s)", flush=True)
    for k, v in res.items():
        print(json.dumps({"variant": k, "best_ms": min(v), "G_evals_s": evals / min(v) / 1e6}), flush=True)


if __name__ == "__main__":
    main()
