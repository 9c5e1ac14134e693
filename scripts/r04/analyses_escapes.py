#!/usr/bin/env python3
"""Round 4 diagnostic: which opcodes the analyses field's paths escape on (bench.run_analyses
with a recording escape handler that drops the state, as the field does without one)."""
import json
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import bench
    from mythril_amd.device import GpuDevice
    from mythril_amd import workloads
    dev = GpuDevice(0)
    out = {}
    for name in (sys.argv[1:] or sorted(workloads.bytecode_names())):
        seen = Counter()

        def handler(state, seen=seen):
            ins = state.environment.code.instruction_list
            pc = state.mstate.pc
            op = ins[pc]["opcode"] if pc < len(ins) else "END"
            st = state.mstate.stack
            tx = state.current_transaction
            top = [("sym" if getattr(x, "symbolic", False) else hex(x.value)) for x in st[-3:][::-1]]
            key = (op, type(tx).__name__, tuple(top), len(state.mstate.memory),
                   bool(state.mstate.memory.symbolic))
            seen[str(key)] += 1
            return []
        bench.run_analyses(dev, 2, 1024, escape_handler=handler, names=[name])
        if seen:
            out[name] = dict(seen)
        print(name, dict(seen), flush=True)
    dev.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
