#!/usr/bin/env python3
"""Per-launch durations of the bench line's headline kernels from a rocprofv3
--kernel-trace CSV of `python bench.py` (the stats file averages every launch of
a kernel, the LaserEVM fields' small in-situ launches included): the C2 batch
launches of k_lane_step (grid = the C2 lanes) and the C4 launches of k_bv_eval
(the largest k_bv_eval grid), with their averages, for comparison with the
line's roofline.kernel_ms.

usage: trace_launches.py <bench_kernel_trace.csv> [c2_lanes] > summary.json"""
import csv
import json
import sys
from collections import defaultdict


def main(path, lanes=65536):
    by = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip()
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        by[(name, grid)].append(dur)
    out = {}
    c2 = [(g, d) for (n, g), d in by.items() if n == "k_lane_step" and g >= lanes]
    if c2:
        g, d = max(c2, key=lambda x: len(x[1]))
        out["k_lane_step_c2"] = {"grid": g, "launches": len(d), "avg_ms": sum(d) / len(d),
                                 "median_ms": sorted(d)[len(d) // 2], "min_ms": min(d)}
    c4 = [(g, d) for (n, g), d in by.items() if n == "k_bv_eval"]
    if c4:
        g, d = max(c4, key=lambda x: x[0])
        out["k_bv_eval_c4"] = {"grid": g, "launches": len(d), "avg_ms": sum(d) / len(d),
                               "median_ms": sorted(d)[len(d) // 2], "min_ms": min(d)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
