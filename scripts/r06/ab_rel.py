"""Interleaved A/B of the exact procedure's first phase (MYTHSMT_REL_BUDGET: the
conflicts a session query is decided on over its own cone before every
variable; 0 = never) on the in-situ bench fields, in one process on one box:

    python scripts/r06/ab_rel.py OUT.json [rounds]

Per round and mode: symbolic_tx (overflow, exceptions; 2 replicas), the
18-contract myth_analyze field (no CPU comparator) and BECToken -t 1, with
their wall and exact-procedure times and the verdict counters, which must not
depend on the mode."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import bench  # noqa: E402
import symref  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402


def one(dev, mode):
    os.environ["MYTHSMT_REL_BUDGET"] = str(mode)
    out = {"mode": mode}
    bench.SYMBOLIC_TX_CODES = ("overflow.sol.o", "exceptions.sol.o")
    st = bench.run_symbolic_tx(dev, 2, 2, 1024, symref.Engine(signals=True).step)
    for n, c in st["contracts"].items():
        out[n] = {"wall_s": c["wall_s"], "exact_ms": c["exact_ms"], "exact": c["exact"],
                  "fork_filter": c["fork_filter"], "open_states": c["open_states"]}
    ma = bench.run_myth_analyze(dev, 2, cpu=False)
    t = ma["totals"]
    out["myth_analyze"] = {"wall_s": t["wall_s"], "exact_s": t["exact_s"], "issues": t["issues"],
                           "unsat": t["unsat_confirmations"], "pruned": t["forks_pruned"]}
    c3 = bench.run_c3_bectoken(dev, 1)["summary"]
    out["c3"] = {k: c3[k] for k in ("wall_s", "exact_s", "exact_calls", "issues", "swc101_at_mul")}
    return out


def main():
    dev = GpuDevice(0)
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    one(dev, 20)                                   # warm-up: compiles, caches, the signature DB
    res = []
    for r in range(rounds):
        for mode in (0, 20):
            t0 = time.perf_counter()
            row = one(dev, mode)
            row["round"], row["total_s"] = r, time.perf_counter() - t0
            res.append(row)
            print(json.dumps(row), flush=True)
    Path(sys.argv[1]).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
