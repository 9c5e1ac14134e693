#!/usr/bin/env python3
"""VALU instructions kernel 2 executes per interpreted 256-bit division, from a
rocprofv3 SQ_INSTS_VALU pass over scripts/k2_opclass.py (every DAG built from
one op class, 4 launches per class in the order the script prints them).

Per class: VALU per wave-instruction = SQ_INSTS_VALU / (instructions x
models / 64).  The divrem and addsub classes differ only in the op of each
level, so a division executes
    VALU/insn(divrem) - VALU/insn(addsub) + 16
VALU instructions (the add's 16 useful int32 ops put back).  Each VALU
instruction is one int32 op per lane, i.e. per constraint-eval, so this is the
division's executed int32-op cost, to set beside the SURVEY §8(d) charge of
32 w^2 = 2,048.

usage: k2_div_valu.py <counter_collection.csv> <k2_opclass stdout log> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict

MODELS = 4096


def main(csv_path, log_path, out_path):
    classes = [json.loads(l) for l in open(log_path) if l.startswith("{")]
    disp = defaultdict(dict)
    for r in csv.DictReader(open(csv_path)):
        if "k_bv_eval" in r["Kernel_Name"]:
            disp[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(disp)
    per = len(ids) // len(classes)
    assert per * len(classes) == len(ids), (len(ids), len(classes))
    out = {"classes": {}}
    for k, c in enumerate(classes):
        vals = [disp[d]["SQ_INSTS_VALU"] for d in ids[k * per:(k + 1) * per]]
        wave_insns = c["insns"] * MODELS / 64
        rec = {"valu_per_wave_insn": sum(vals) / len(vals) / wave_insns, "insns": c["insns"]}
        for name in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM"):
            if name in disp[ids[k * per]]:
                rec[name.lower().replace("sq_insts_", "") + "_per_wave_insn"] = \
                    disp[ids[k * per]][name] / wave_insns
        out["classes"][c["class"]] = rec
    div = out["classes"]["divrem"]["valu_per_wave_insn"]
    add = out["classes"]["addsub"]["valu_per_wave_insn"]
    out["valu_per_division"] = div - add + 16.0
    out["survey_charge_per_division"] = 2048.0
    out["source"] = f"{csv_path} + {log_path}"
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps({"valu_per_division": out["valu_per_division"],
                      "per_class": {k: round(v["valu_per_wave_insn"], 1) for k, v in out["classes"].items()}}))


if __name__ == "__main__":
    main(*sys.argv[1:4])
