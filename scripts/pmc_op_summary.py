#!/usr/bin/env python3
"""Per-pattern SQ instruction counts per wave of kernel 1 (scripts/archive/gpu_pmc_op.sh)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
for d in sorted(src.glob("pmcop_*")):
    f = d / "run_counter_collection.csv"
    if not f.exists():
        continue
    acc = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_lane_step" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
    w = acc.get("SQ_WAVES", 0) or 1
    print(d.name[6:], " ".join(f"{k[3:]}={v / w:.0f}" for k, v in sorted(acc.items()) if k != "SQ_WAVES"))
