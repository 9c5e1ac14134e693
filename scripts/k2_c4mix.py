#!/usr/bin/env python3
"""Kernel 2 on the C4 op mix only (65,536 DAGs x 4,096 models, 3 timed runs):
the short, fixed workload behind the rocprofv3 counter passes of kernel-2
A/Bs (scripts/archive/gpu_r02c.sh).  Prints ms per launch and G constraint-evals/s."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.smt import synth  # noqa: E402

N = 1 << 16


def main():
    dev = GpuDevice(0)
    models = synth.c4_models(4096, synth.C4_SEED + 0x1000)
    prog = synth.c4_programs(synth.Draws(N, synth.C4_SEED))
    dev.eval_upload(prog, models)
    dev.eval_run()
    ms = [dev.eval_run() for _ in range(3)]
    fs, sc = dev.eval_download()
    print(json.dumps({"ms": min(ms), "G_evals_s": N * 4096 / min(ms) / 1e6,
                      "sat_dags": int((sc > 0).sum()), "sat_total": int(sc.sum())}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
