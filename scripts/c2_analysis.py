#!/usr/bin/env python3
"""Where kernel 1's C2 time goes, estimated on the CPU oracle (no GPU needed):
per-lane path lengths, per-wave opcode-group iterations of the device's
dispatch (one iteration runs all live lanes whose next opcode equals the lowest
live lane's), and how many steps take the general (slow) handler."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from mythril_amd import workloads  # noqa: E402
from mythril_amd.lanes import MG_RUNNING, bucket_order, permuted  # noqa: E402
from oracle.evm_ref import OracleEVM  # noqa: E402

FAST_KINDS = {"push", "dup", "swap", "pop", "jumpdest", "jump", "jumpi", "alu", "env", "mload",
              "mstore", "cdload"}


def kind(op):
    if 0x60 <= op <= 0x7F: return "push"
    if 0x80 <= op <= 0x8F: return "dup"
    if 0x90 <= op <= 0x9F: return "swap"
    if op == 0x50: return "pop"
    if op == 0x5B: return "jumpdest"
    if op == 0x56: return "jump"
    if op == 0x57: return "jumpi"
    if op <= 0x03 or op == 0x0B or 0x10 <= op <= 0x1D: return "alu"
    if op in (0x30, 0x32, 0x33, 0x34, 0x36, 0x38, 0x3A, 0x3D, 0x45, 0x58, 0x59): return "env"
    if op == 0x51: return "mload"
    if op == 0x52: return "mstore"
    if op == 0x35: return "cdload"
    return "slow"


def main(n=65536):
    code = workloads.bytecode("overflow.sol.o")
    b = workloads.c2_batch(n, stack_cap=64, mem_cap=1024)
    b = permuted(b, bucket_order(b))
    o = OracleEVM()
    cid = o.load_code(code)
    b.code_id[:] = cid
    ops, _ = o.code_table(cid)
    ops = ops.astype(np.int32)
    hist = []                      # per round: opcode of each live lane (-1 if not live)
    while True:
        live = b.status == MG_RUNNING
        if not live.any():
            break
        pc = b.pc.astype(np.int64)
        cur = np.where(live & (pc < ops.size), ops[np.minimum(pc, ops.size - 1)], -1)
        hist.append(cur.astype(np.int32))
        o.run(b, max_steps=1)
    H = np.stack(hist)                              # rounds x lanes
    steps = (H >= 0).sum(0)
    print(f"lanes {n}  rounds {H.shape[0]}  steps/lane mean {steps.mean():.1f} "
          f"p50 {np.median(steps):.0f} p99 {np.percentile(steps, 99):.0f} max {steps.max()}")
    kinds = np.vectorize(kind)(np.maximum(H, 0))
    slow = ((kinds == "slow") & (H >= 0)).sum()
    print(f"slow-handler opcodes: {slow / (H >= 0).sum():.1%} of steps, {slow / n:.1f} per lane")
    # opcode-merge simulation per wave
    iters = []
    for w in range(0, n, 64):
        seqs = [list(H[:, l][H[:, l] >= 0]) for l in range(w, min(w + 64, n))]
        pos = [0] * len(seqs)
        it = 0
        while True:
            live = [i for i in range(len(seqs)) if pos[i] < len(seqs[i])]
            if not live:
                break
            op = seqs[live[0]][pos[live[0]]]
            for i in live:
                if seqs[i][pos[i]] == op:
                    pos[i] += 1
            it += 1
        iters.append(it)
    iters = np.array(iters)
    wave_max = np.array([steps[w:w + 64].max() for w in range(0, n, 64)])
    print(f"wave iterations mean {iters.mean():.0f} max {iters.max()}  "
          f"(longest lane per wave mean {wave_max.mean():.0f}); divergence x{iters.mean() / wave_max.mean():.2f}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 65536)


def histogram(n=8192):
    from mythril_amd.laser.opcodes import ADDRESS_OPCODE_MAPPING
    code = workloads.bytecode("overflow.sol.o")
    b = workloads.c2_batch(n, stack_cap=64, mem_cap=1024)
    o = OracleEVM()
    cid = o.load_code(code)
    b.code_id[:] = cid
    ops, _ = o.code_table(cid)
    ops = ops.astype(np.int32)
    cnt = np.zeros(256, dtype=np.int64)
    depth_hist = np.zeros(1025, dtype=np.int64)
    while True:
        live = b.status == MG_RUNNING
        if not live.any():
            break
        pc = b.pc.astype(np.int64)
        ok = live & (pc < ops.size)
        np.add.at(cnt, ops[pc[ok]], 1)
        np.add.at(depth_hist, b.sp[ok].astype(np.int64), 1)
        o.run(b, max_steps=1)
    tot = cnt.sum()
    for op in np.argsort(-cnt)[:25]:
        print(f"  {ADDRESS_OPCODE_MAPPING.get(int(op), hex(op)):10s} {cnt[op] / n:7.2f}/lane  {cnt[op] / tot:6.1%}")
    d = np.nonzero(depth_hist)[0]
    print("stack depth at step: max", d.max(), " share >= 14:", depth_hist[14:].sum() / tot)
