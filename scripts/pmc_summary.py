#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from rocprofv3 --pmc passes.

Reads the FETCH_SIZE and WRITE_SIZE passes (separate runs, see
scripts/archive/gpu_check.sh) and writes <out>/traffic.json:
  {kernel: {"fetch_bytes": F, "write_bytes": W, "traffic_bytes": F + W, "launches": n}}
Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): both counters are in
KiB; on gfx950 FETCH_SIZE reports half of the bytes of a wide coalesced read,
so it is doubled; WRITE_SIZE is taken as is.  bench.py reports traffic_bytes of
the dominant kernel as roofline.traffic.

usage: python scripts/pmc_summary.py gpurun_out profiles/r01
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def per_kernel(path: Path, counter: str):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            name = name.removeprefix("void ").split("<")[0].strip()
            acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main(src: str, dst: str):
    src_p, dst_p = Path(src), Path(dst)
    fetch = per_kernel(src_p / "prof_fetch" / "run_counter_collection.csv", "FETCH_SIZE")
    write = per_kernel(src_p / "prof_write" / "run_counter_collection.csv", "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = 2.0 * fetch.get(k, (0.0, 0))[0]
        w = write.get(k, (0.0, 0))[0]
        out[k] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w,
                  "launches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
    dst_p.mkdir(parents=True, exist_ok=True)
    (dst_p / "traffic.json").write_text(json.dumps(out, indent=1) + "\n")
    for k, v in out.items():
        print(f"{k:28s} fetch {v['fetch_bytes'] / 1e6:10.2f} MB  write {v['write_bytes'] / 1e6:10.2f} MB")


if __name__ == "__main__":
    main(*(sys.argv[1:3] if len(sys.argv) >= 3 else ("gpurun_out", "profiles/r01")))
