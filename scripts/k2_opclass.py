#!/usr/bin/env python3
"""Kernel 2 time per C4 op class: every DAG's 32 levels use one class (same
draws otherwise), 65,536 DAGs x 4096 models; prints ms, evals/s and the
§8(d) algorithmic int32-op rate per class next to the real C4 mix."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.smt import synth  # noqa: E402

N = 1 << 16
NAMES = ["addsub", "logic", "mul", "shift", "extcat", "ite", "cmp", "divrem"]


def run(dev, prog, models, reps=3):
    dev.eval_upload(prog, models)
    dev.eval_run()
    ms = min(dev.eval_run() for _ in range(reps))
    ops = synth.program_cost(prog)[0]
    return ms, ops


def main():
    dev = GpuDevice(0)
    models = synth.c4_models(4096, synth.C4_SEED + 0x1000)
    out = {}
    dr = synth.Draws(N, synth.C4_SEED)
    ms, ops = run(dev, synth.c4_programs(dr), models)
    out["c4_mix"] = ms
    print(json.dumps({"class": "c4_mix", "ms": ms, "G_evals_s": N * 4096 / ms / 1e6,
                      "T_ops_s": ops * 4096 / ms / 1e9, "insns": int(synth.c4_programs(dr).prog_off[-1])}), flush=True)
    for k, name in enumerate(NAMES):
        dr = synth.Draws(N, synth.C4_SEED)
        dr.cls[:] = k
        prog = synth.c4_programs(dr)
        ms, ops = run(dev, prog, models)
        print(json.dumps({"class": name, "ms": ms, "G_evals_s": N * 4096 / ms / 1e6,
                          "T_ops_s": ops * 4096 / ms / 1e9, "insns": int(prog.prog_off[-1])}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
