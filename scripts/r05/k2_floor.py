#!/usr/bin/env python3
"""Kernel 2's issue-bound floor per op class: the SQ
pass of scripts/k2_opclass.py (gpurun_out/r05*/k2sq) gives, per launch, the
wave-instructions each class issues; the issue-rate probe
(scripts/probes/issue_rates.hip, profiles/r05/issue_rates.json) gives how many
of each class one CU issues per clock at 8 waves per SIMD.  The floor of a
launch is the largest class time (instructions per CU / rate / clock); the
kernel's measured time over it is how close it runs to issue-bound.

usage: python scripts/r05/k2_floor.py <k2sq dir> <issue_rates.json> <k2sq.log> [out.json]"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

CLK = 2.4e9
CUS = 256


def main(sqdir, rates_path, log_path, out=None):
    rates = json.loads(Path(rates_path).read_text())["rates"]
    salu = rates["salu"]["8"]["wave_instr_per_cu_clk"] * 19.0 / 16.0   # + the loop's 3 SALU/branch
    valu = rates["valu"]["8"]["wave_instr_per_cu_clk"]
    branch = rates["branch"]["8"]["wave_instr_per_cu_clk"]             # s_cmp + s_cbranch pairs
    rows = defaultdict(dict)
    for f in Path(sqdir).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "k_bv_eval" not in r["Kernel_Name"]:
                continue
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    classes = [json.loads(l) for l in Path(log_path).read_text().splitlines() if l.startswith("{")]
    disp = sorted(rows)
    # k2_opclass.py: per class one warm-up launch then 3 timed ones (run()); keep the last of each group
    per = len(disp) // max(len(classes), 1)
    res = {}
    for k, c in enumerate(classes):
        d = rows[disp[(k + 1) * per - 1]]
        w = d["SQ_WAVES"]
        s, v, b = d["SQ_INSTS_SALU"], d["SQ_INSTS_VALU"], d["SQ_INSTS_BRANCH"]
        t_s = s / CUS / salu / CLK * 1e3
        t_v = v / CUS / valu / CLK * 1e3
        t_b = 2.0 * b / CUS / branch / CLK * 1e3
        floor = max(t_s, t_v, t_b)
        res[c["class"]] = {"ms": c["ms"], "waves": w, "salu_per_wave": s / w, "valu_per_wave": v / w,
                           "branch_per_wave": b / w, "insns": c["insns"],
                           "salu_per_insn": s / (c["insns"] * 4096 / 64), "valu_per_insn": v / (c["insns"] * 4096 / 64),
                           "floor_ms": {"salu": t_s, "valu": t_v, "branch": t_b}, "bound": max(
                               (("salu", t_s), ("valu", t_v), ("branch", t_b)), key=lambda x: x[1])[0],
                           "frac_of_floor": floor / c["ms"],
                           "wait_any_frac": d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"],
                           "issue_stall_frac": d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]}
    txt = json.dumps({"rates_per_cu_clk": {"salu": salu, "valu": valu, "branch_pairs": branch},
                      "classes": res}, indent=1)
    print(txt)
    if out:
        Path(out).write_text(txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
