import sys; from pathlib import Path; sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np, collections
from mythril_amd import workloads
from oracle.evm_ref import OracleEVM
from mythril_amd.lanes import MG_RUNNING
b = workloads.c2_batch(2048, stack_cap=64, mem_cap=1024)
o = OracleEVM(); cid = o.load_code(workloads.bytecode("overflow.sol.o")); b.code_id[:] = cid
ops, _ = o.code_table(cid)
h = collections.Counter(); sps = collections.Counter()
for r in range(400):
    live = np.nonzero(b.status == MG_RUNNING)[0]
    if live.size == 0: break
    for i in live:
        pc = int(b.pc[i])
        if pc < ops.size:
            h[int(ops[pc])] += 1
            sps[min(int(b.sp[i]), 20)] += 1
    o.run(b, max_steps=1)
tot = sum(h.values())
names = {0x51:"MLOAD",0x52:"MSTORE",0x35:"CDLOAD",0x54:"SLOAD",0x55:"SSTORE",0x20:"SHA3",0x56:"JUMP",0x57:"JUMPI",0x5b:"JUMPDEST",0x50:"POP"}
for op, c in h.most_common(40):
    n = names.get(op, hex(op))
    print(f"{n:10s} {c/tot*100:6.2f}%")
print("sp dist", sorted(sps.items()))
