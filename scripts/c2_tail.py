#!/usr/bin/env python3
"""Opcode mix of the C2 lanes that set kernel 1's launch time (the longest
paths), next to the mix of all lanes (CPU oracle, no GPU needed)."""
import collections
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

from mythril_amd import workloads  # noqa: E402
from mythril_amd.lanes import MG_RUNNING  # noqa: E402
from oracle.evm_ref import OracleEVM  # noqa: E402


def main(n=2048, tail=190):
    b = workloads.c2_batch(n, stack_cap=64, mem_cap=1024)
    o = OracleEVM()
    cid = o.load_code(workloads.bytecode("overflow.sol.o"))
    b.code_id[:] = cid
    ops, _ = o.code_table(cid)
    seq = [[] for _ in range(n)]
    for _ in range(400):
        live = np.nonzero(b.status == MG_RUNNING)[0]
        if live.size == 0:
            break
        for i in live:
            pc = int(b.pc[i])
            if pc < ops.size:
                seq[i].append(int(ops[pc]))
        o.run(b, max_steps=1)
    long_ = [s for s in seq if len(s) >= tail]
    print(f"lanes {n}, tail lanes (>= {tail} steps): {len(long_)}")
    for name, group in (("tail", long_), ("all", seq)):
        h = collections.Counter(op for s in group for op in s)
        tot = sum(h.values())
        print(name, " ".join(f"{op:02x}:{c / len(group):.1f}" for op, c in h.most_common(30)))


if __name__ == "__main__":
    main()
