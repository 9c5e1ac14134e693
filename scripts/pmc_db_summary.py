#!/usr/bin/env python3
"""Per-wave averages of SQ counters from rocprofv3 SQLite outputs (pmc_results.db):
usage: pmc_db_summary.py KERNEL_SUBSTRING name=dir1,dir2 [name=...]"""
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path


def collect(dirs, kern):
    acc = defaultdict(list)
    dur = []
    for d in dirs:
        for db in Path(d).glob("**/*.db"):
            c = sqlite3.connect(str(db))
            for name, val, kn, du in c.execute(
                    "select counter_name, value, kernel_name, duration from counters_collection"):
                if kern in kn:
                    acc[name].append(float(val))
                    dur.append(float(du))
    return {k: sum(v) / len(v) for k, v in acc.items()}, (sum(dur) / len(dur) if dur else 0)


def main():
    kern = sys.argv[1]
    for arg in sys.argv[2:]:
        name, dirs = arg.split("=")
        d, du = collect(dirs.split(","), kern)
        w = d.get("SQ_WAVES", 1.0)
        print(f"{name}: dispatch {du / 1e3:.1f} us, waves {w:.0f}")
        for k in sorted(d):
            print(f"   {k:22s} total {d[k]:16.0f}   per wave {d[k] / w:12.1f}")


if __name__ == "__main__":
    main()
