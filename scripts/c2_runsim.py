#!/usr/bin/env python3
"""Iterations kernel 1's dispatch loop needs per wave on C2 (CPU oracle):
a straight-line run (mg_load_code's run table) advances every lane at the lead
lane's pc; any other step advances the lanes whose next opcode equals the
lead's.  Reports iterations per wave against the longest lane per wave."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

from mythril_amd import workloads  # noqa: E402
from mythril_amd.lanes import MG_RUNNING, bucket_order, permuted  # noqa: E402
from oracle.evm_ref import OracleEVM  # noqa: E402

RUN_MAX = 64


def simple(b):
    return (0x60 <= b <= 0x7F or 0x80 <= b <= 0x9F or b in (0x50, 0x5B, 0x15, 0x19)
            or 0x01 <= b <= 0x03 or b == 0x0B or 0x10 <= b <= 0x1D)


def run_table(ops):
    n = len(ops)
    ln = [0] * (n + 1)
    for i in range(n - 1, -1, -1):
        if simple(int(ops[i])):
            cont = 0 < ln[i + 1] < RUN_MAX
            ln[i] = 1 + (ln[i + 1] if cont else 0)
    return ln


def main(n=8192):
    b = workloads.c2_batch(n, stack_cap=64, mem_cap=1024)
    b = permuted(b, bucket_order(b))
    o = OracleEVM()
    cid = o.load_code(workloads.bytecode("overflow.sol.o"))
    b.code_id[:] = cid
    ops, _ = o.code_table(cid)
    rl = run_table(ops)
    rows = []
    while True:
        live = b.status == MG_RUNNING
        if not live.any():
            break
        rows.append(np.where(live & (b.pc < ops.size), b.pc.astype(np.int64), -1))
        o.run(b, max_steps=1)
    P = np.stack(rows)
    steps = (P >= 0).sum(0)
    it_all, runs_all, single_all, wmax = [], [], [], []
    for w in range(0, n, 64):
        seqs = [P[:, l][P[:, l] >= 0] for l in range(w, min(w + 64, n))]
        pos = [0] * len(seqs)
        it = runs = single = 0
        while True:
            live = [i for i in range(len(seqs)) if pos[i] < len(seqs[i])]
            if not live:
                break
            pc0 = int(seqs[live[0]][pos[live[0]]])
            it += 1
            if rl[pc0] >= 2:
                runs += 1
                for i in live:
                    if int(seqs[i][pos[i]]) == pc0:
                        pos[i] = min(pos[i] + rl[pc0], len(seqs[i]))
            else:
                single += 1
                op0 = int(ops[pc0])
                for i in live:
                    if int(ops[int(seqs[i][pos[i]])]) == op0:
                        pos[i] += 1
        it_all.append(it); runs_all.append(runs); single_all.append(single)
        wmax.append(int(max(len(s) for s in seqs)))
    it_all, wmax = np.array(it_all), np.array(wmax)
    k = int(np.argmax(it_all))
    print(f"lanes {n}: steps/lane mean {steps.mean():.1f} max {steps.max()}")
    print(f"iterations/wave mean {it_all.mean():.1f} max {it_all.max()} "
          f"(runs {runs_all[k]}, single {single_all[k]} in the max wave; its longest lane {wmax[k]})")
    print(f"longest lane per wave mean {wmax.mean():.1f}; iterations per longest-lane step "
          f"{(it_all / wmax).mean():.2f}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8192)
