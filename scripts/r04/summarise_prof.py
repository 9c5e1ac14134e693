#!/usr/bin/env python3
"""Summaries of the round-4 profiling job (scripts/r04/gpu_prof.sh) for
profiles/r04/: per-launch HBM traffic (FETCH_SIZE x2 on gfx950, KiB -> bytes;
MI355X_MICROARCH.md HBM/rocprofv3 section) of k_bv_eval (C4) and of k_sym_step's
timed launches (symbolic / taint separately), and the SQ counters per wave.

usage: python scripts/r04/summarise_prof.py gpurun_out/r04c profiles/r04"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path


def counters(d: Path):
    f = glob.glob(str(d / "**" / "run_counter_collection.csv"), recursive=True)[0]
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].removeprefix("void ").split("<")[0].strip()
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def mean(v):
    return sum(v) / len(v)


def main(src: str, dst: str):
    s, d = Path(src), Path(dst)
    d.mkdir(parents=True, exist_ok=True)
    traffic = {}
    for kernel, fdir, wdir, what in (
            ("k_bv_eval", "k2_fetch", "k2_write", "scripts/r03/k2_c4.py: the bench's C4 batch, 2 launches"),
            ("k_sym_step", "sym_symbolic_fetch", "sym_symbolic_write",
             "scripts/r04/sym_timed.py symbolic: the symbolic_lanes field's 6 timed launches, no profiling pass")):
        f = counters(s / fdir)[kernel]["FETCH_SIZE"]
        w = counters(s / wdir)[kernel]["WRITE_SIZE"]
        fb, wb = 2.0 * mean(f) * 1024.0, mean(w) * 1024.0
        traffic[kernel] = {"fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb, "launches": len(f),
                           "command": what}
    f = counters(s / "sym_taint_fetch")["k_sym_step"]["FETCH_SIZE"]
    w = counters(s / "sym_taint_write")["k_sym_step"]["WRITE_SIZE"]
    taint = {"fetch_bytes": 2.0 * mean(f) * 1024.0, "write_bytes": mean(w) * 1024.0, "launches": len(f),
             "command": "scripts/r04/sym_timed.py taint: the taint_lanes field's 6 launches"}
    taint["traffic_bytes"] = taint["fetch_bytes"] + taint["write_bytes"]
    traffic["_source"] = {"job": f"{src} (scripts/r04/gpu_prof.sh)", "correction": "FETCH_SIZE x2 on gfx950, KiB",
                          "k_sym_step_taint_lanes": taint}
    (d / "traffic.json").write_text(json.dumps(traffic, indent=1) + "\n")
    sq = {}
    for name, a, b in (("k_bv_eval", "k2_sq_a", "k2_sq_b"), ("k_lane_step", "k1_sq_a", "k1_sq_b")):
        c = {**counters(s / a)[name], **counters(s / b)[name]}
        waves = mean(c["SQ_WAVES"])
        per = {k: mean(v) / waves for k, v in c.items() if k != "SQ_WAVES"}
        per["SQ_WAVES"] = waves
        per["wait_any_frac"] = mean(c["SQ_WAIT_ANY"]) / mean(c["SQ_WAVE_CYCLES"])
        per["wait_inst_frac"] = mean(c["SQ_WAIT_INST_ANY"]) / mean(c["SQ_WAVE_CYCLES"])
        sq[name] = per
    (d / "sq_per_wave.json").write_text(json.dumps(sq, indent=1) + "\n")
    print(json.dumps(traffic, indent=1))
    print(json.dumps(sq, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
