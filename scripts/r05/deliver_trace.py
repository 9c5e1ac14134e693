"""Round 5 diagnostic: the device events LaserEVM._deliver receives during
myth analyze -f <code> -t 2 -m <module> (status, aux, pc, address, lane flags)."""
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import analyze  # noqa: E402
import fnames  # noqa: E402
from mythril_amd.laser import svm  # noqa: E402
from mythril_amd.laser.disassembly import SignatureDB  # noqa: E402
from oracle_device import OracleDevice, OracleK2  # noqa: E402

name, module = sys.argv[1], sys.argv[2]
d = tempfile.mkdtemp()
fnames.signature_db(Path(d))
os.environ["MYTHRIL_DIR"] = d
SignatureDB._reset()
orig = svm.LaserEVM._deliver


def deliver(self, ln, b, *a, **k):
    i = ln.pos
    pc = int(b.pc[i])
    ins = ln.state.environment.code.instruction_list
    addr = ins[pc]["address"] if pc < len(ins) else None
    print("  ev", int(b.status[i]), hex(int(b.aux[i])), "pc", pc, "addr", addr,
          ins[pc]["opcode"] if pc < len(ins) else None, "flags", hex(int(b.flags[i])), "sp", int(b.sp[i]),
          flush=True)
    return orig(self, ln, b, *a, **k)


svm.LaserEVM._deliver = deliver
import symref  # noqa: E402
ostep = symref.Engine.step


def step(self, state):
    ms = state.mstate
    ins = state.environment.code.instruction_list
    op = ins[ms.pc]["opcode"] if ms.pc < len(ins) else None
    try:
        out = ostep(self, state)
    except Exception as e:  # noqa: BLE001 -- printed and re-raised
        print("  esc", op, "pc", ms.pc, "raised", type(e).__name__, str(e)[:200],
              [repr(w)[:60] for w in ms.stack[-4:]], flush=True)
        raise
    print("  esc", op, "pc", ms.pc, "->", len(out), flush=True)
    if op in ("CODECOPY", "CODESIZE", "CALLDATACOPY"):
        print("   in:", [repr(w)[:50] for w in ms.stack[-4:]], type(state.environment.calldata).__name__,
              type(state.current_transaction).__name__, "msize", len(ms.memory),
              "out memsym", [o.mstate.memory.symbolic for o in out], flush=True)
    return out


symref.Engine.step = step
opack = svm.LaserEVM._pack


def pack(self, b, i, st):
    opack(self, b, i, st)
    print("  pack", i, "pc", st.mstate.pc, "flags", hex(int(b.flags[i])), "memsym", st.mstate.memory.symbolic,
          "symbatch", b.symbolic, flush=True)


svm.LaserEVM._pack = pack
if "--gpu" in sys.argv:
    from mythril_amd.device import GpuDevice
    dev = k2 = GpuDevice(0)
else:
    dev, k2 = OracleDevice(), OracleK2()
issues, info = analyze.analyze(name, module, 2, dev, k2)
print(analyze.issue_table(issues), {k: info[k] for k in ("lane_steps", "launches", "forks", "escapes_dropped")})
