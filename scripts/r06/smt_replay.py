"""Replay dumped exact-procedure queries (MYTHSMT_DUMP=dir) against
libmythsmt.so: per query the verdict, wall time and CNF size -- the A/B
harness for the bit-blaster and the CDCL core.

    python scripts/r06/smt_replay.py <dir> [max_ms]
"""
import ctypes
import glob
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from mythril_amd.smt import exact  # noqa: E402


def main():
    d = sys.argv[1]
    max_ms = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    lib = exact.load()
    tot = 0.0
    verdicts = {}
    for f in sorted(glob.glob(f"{d}/*.npz")):
        z = np.load(f)
        nodes, args, limbs, roots, mins, counts = (z[k] for k in ("nodes", "args", "limbs", "roots", "mins", "counts"))
        roots_a = roots if roots.size else np.zeros(1, np.uint32)
        mins_a = mins if mins.size else np.zeros(1, np.uint32)
        q = exact.MsQuery(nodes.size // 6, nodes.ctypes.data, args.ctypes.data, limbs.ctypes.data, roots.size,
                          roots_a.ctypes.data, mins.size, mins_a.ctypes.data, int(counts[0]), int(counts[1]),
                          int(counts[2]))
        lim = exact.MsLimits(0, max_ms, 2000)
        st = exact.MsStats()
        out = np.zeros(1 << 20, dtype=np.uint32)
        n = ctypes.c_uint32(0)
        t0 = time.perf_counter()
        rc = lib.ms_solve(ctypes.byref(q), ctypes.byref(lim), out.ctypes.data, out.size, ctypes.byref(n),
                          ctypes.byref(st))
        el = time.perf_counter() - t0
        tot += el
        verdicts[Path(f).name] = rc
        print(f"{Path(f).name} rc={rc} {el * 1e3:8.1f} ms nodes={nodes.size // 6} vars={st.vars} "
              f"clauses={st.clauses} conflicts={st.conflicts} mins={mins.size}", flush=True)
    print(f"total {tot:.2f} s; sat {sum(v == 1 for v in verdicts.values())} unsat "
          f"{sum(v == 0 for v in verdicts.values())} unknown {sum(v == 2 for v in verdicts.values())}")


if __name__ == "__main__":
    main()
