#!/usr/bin/env python3
"""Per-kernel averages of the SQ counter passes written by scripts/archive/gpu_pmc.sh."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(src.glob("pmc_sq*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if k.startswith("k_lane_step") or k.startswith("k_bv_eval"):
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(avg):
        print(f"  {c:24s} {avg[c]:16.0f}")
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        print(f"  VALU insts/wave          {avg['SQ_INSTS_VALU'] / avg['SQ_WAVES']:16.0f}")
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_BUSY_CYCLES" in avg:
        # SQ_ACTIVE_INST_VALU counts quad-cycles summed over SIMDs of an SE (see guide)
        print(f"  ACTIVE_VALU/BUSY         {avg['SQ_ACTIVE_INST_VALU'] / avg['SQ_BUSY_CYCLES']:16.3f}")
