"""Interleaved A/B of an exact-procedure switch on the in-situ bench fields, in
one process on one box (the switches are read at every solve):

    python scripts/r06/ab_rel.py OUT.json [rounds] [VAR v1,v2] [codes]

VAR defaults to MYTHSMT_REL_BUDGET 0,20 (the conflicts a session query is
decided on over its own cone before every variable; 0 = never); MYTHSMT_EAGER
0,1 is the eager small-domain congruence.  codes: the symbolic_tx contracts
(default overflow.sol.o,exceptions.sol.o).

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


VAR, MODES, CODES = "MYTHSMT_REL_BUDGET", ("0", "20"), ("overflow.sol.o", "exceptions.sol.o")


def one(dev, mode):
    os.environ[VAR] = str(mode)
    out = {"var": VAR, "mode": mode}
    bench.SYMBOLIC_TX_CODES = CODES
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
    global VAR, MODES, CODES
    dev = GpuDevice(0)
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    if len(sys.argv) > 4:
        VAR, MODES = sys.argv[3], tuple(sys.argv[4].split(","))
    if len(sys.argv) > 5:
        CODES = tuple(sys.argv[5].split(","))
    one(dev, MODES[-1])                            # warm-up: compiles, caches, the signature DB
    res = []
    for r in range(rounds):
        for mode in MODES:
            t0 = time.perf_counter()
            row = one(dev, mode)
            row["round"], row["total_s"] = r, time.perf_counter() - t0
            res.append(row)
            print(json.dumps(row), flush=True)
    Path(sys.argv[1]).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
