#!/usr/bin/env python3
"""Kernel 2 on the bench's C4 batch (1M DAGs x 4,096 models), two launches:
the command the per-launch PMC passes (FETCH_SIZE / WRITE_SIZE / SQ_*) profile."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    from mythril_amd.device import GpuDevice
    from mythril_amd.smt import synth
    prog, models = synth.c4_batch(1_000_000, 4096)
    dev = GpuDevice(0)
    dev.eval_upload(prog, models)
    ms = [dev.eval_run() for _ in range(2)]
    print(json.dumps({"ms": ms}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
