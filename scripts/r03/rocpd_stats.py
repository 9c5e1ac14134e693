#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 rocpd database (run_results.db,
the default output format of rocprofv3 here): calls, average, min, max and
every duration of the kernels matching a filter.
usage: rocpd_stats.py <run_results.db> [substring ...]"""
import sqlite3
import sys
from collections import defaultdict


def main(path, keys):
    db = sqlite3.connect(path)
    cur = db.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch_"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol_"))
    rows = cur.execute(f"select k.kernel_name, d.start, d.end from {disp} d join {sym} k "
                       f"on d.kernel_id = k.id order by d.start").fetchall()
    acc = defaultdict(list)
    for name, a, b in rows:
        acc[name.split("(")[0]].append((b - a) / 1e3)
    print(f"{'kernel':44s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s}")
    for name, v in sorted(acc.items(), key=lambda x: -sum(x[1])):
        if keys and not any(k in name for k in keys):
            continue
        print(f"{name[:44]:44s} {len(v):6d} {sum(v) / len(v):10.2f} {min(v):10.2f} {max(v):10.2f}")
        if keys:
            print("    " + " ".join(f"{x:.2f}" for x in v))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
