"""Taint lanes on an MI355X: k_sym_step's object handles and
annotation masks against the object-level restatement (tests/taintref.py,
values from the C oracle).

* device planes: C2 lanes plus crafted codes (DUP aliasing of an annotated
  word, SWAP, environment objects annotated through ADD and ORIGIN, EXP's early
  return, zero divisors and BYTE, a JUMPI yield on a yield-class atom, the
  64-atom limit, handle compaction with a tiny object table) run under the
  integer + TxOrigin action words; statuses, pcs, steps, gas, the record logs
  word for word, atom counts, sink and yield masks, and per lane the partition
  of stack slots into objects with each slot's atom set must equal the
  restatement's (handle numbers are the device's own);
* end to end: LaserEVM on the GPU with the restated integer and TxOrigin
  modules ends every path with the same annotations, state annotations and
  issues whether their hooks run as device actions or on the host.
"""
import numpy as np
import pytest

from mythril_amd import workloads
from mythril_amd.device import GpuDevice
from mythril_amd.lanes import (MG_ENV_WORDS, MG_LANE_TAINT, MG_TAINT_OBJ0, LaneBatch, LaneShape,
                               word_to_limbs)
from mythril_amd.laser import BreadthFirstSearchStrategy, DepthFirstSearchStrategy
from mythril_amd.laser.opcodes import OPCODES
from oracle_device import OracleDevice

pytestmark = pytest.mark.gpu

# integer module (ADD/MUL/SUB annotate operand 0, EXP with its early return,
# SSTORE/JUMPI sinks) + TxOrigin (ORIGIN post annotation in the yield class,
# JUMPI yields on it): what TaintPlan builds for them (test_taint_cpu.py)
ACTIONS = np.zeros(256, dtype=np.uint32)
for _op in ("ADD", "MUL", "SUB"):
    ACTIONS[OPCODES[_op]] = 1
ACTIONS[OPCODES["EXP"]] = 1 | 32
ACTIONS[OPCODES["SSTORE"]] = 2 << 8
ACTIONS[OPCODES["JUMPI"]] = (2 << 8) | (2 << 12)
ACTIONS[OPCODES["ORIGIN"]] = 16 | 64
# deferred hooks (ArbitraryStorage SSTORE, UserAssertions MSTORE, Exceptions JUMP),
# ArbitraryJump's if-symbolic JUMP/JUMPI, StateChangeAfterCall's if-annotation SLOAD
ACTIONS[OPCODES["SSTORE"]] |= 1 << 16
ACTIONS[OPCODES["MSTORE"]] = 2 << 16
ACTIONS[OPCODES["JUMP"]] = (1 << 16) | (1 << 20)
ACTIONS[OPCODES["JUMPI"]] |= 1 << 20
ACTIONS[OPCODES["SLOAD"]] = 1 << 24

CRAFTED = [
    # PUSH 3, PUSH 5, DUP2, ADD (annotates the DUP'd 3: slot 0 too), PUSH 0, SSTORE, STOP
    "600360058101600055" + "00",
    # ORIGIN (post atom, yield class), PUSH 0, EQ, PUSH 7, JUMPI: yields; JUMPDEST STOP
    "32600014600757" + "5b00",
    # CALLER, PUSH 1, SWAP1, ADD (annotates the environment's caller object), POP,
    # CALLER, CALLER, ADD, ADDRESS, CALLVALUE, MUL, CALLDATASIZE, GASPRICE, SUB, STOP
    "33600190015033330130340236" + "3a03" + "00",
    # EXP 10**2 (annotated), EXP 1**0 and 0**5 (the early return), STOP
    "6002600a0a" + "600060010a" + "600560000a" + "00",
    # annotated 7 DIV 0 (fresh), annotated 9 MOD 3 (union), BYTE 31 / BYTE 40 of it
    "6000600160060104" + "80" + "6003600860010106" + "80601f1a" + "9060281a" + "00",
    # ADDMOD / MULMOD / ISZERO / NOT / LT / SHL over annotated words
    "6001600101" + "6002600201" + "600508" + "8080600709" + "15" + "19" + "8010" + "60031b" + "00",
    # ADDs in a loop while 70 > x: the 64-atom limit (MG_ESC_TAINT)
    "6000" + "5b" + "600101" + "80" + "604611" + "600257" + "00",
    # PUSH/DUP/POP/POP loop: one new handle per round, compaction with a small
    # object table, then out of gas
    "5b" + "6007" + "80" + "5050" + "600056",
]



def _batch(n_c2=48, obj_cap=64):
    c2 = workloads.c2_batch(n_c2, seed=5, stack_cap=64, mem_cap=1024)
    n = n_c2 + 2 * len(CRAFTED)
    b = LaneBatch(LaneShape(n=n, stack_cap=64, mem_cap=1024, calldata_cap=c2.shape.calldata_cap,
                            storage_cap=16, rec_cap=2048, obj_cap=obj_cap))
    codes = [workloads.bytecode("overflow.sol.o")] + [bytes.fromhex(h) for h in CRAFTED]
    for i in range(n_c2):
        for f in ("pc", "sp", "msize", "depth", "status", "aux", "steps", "flags", "calldata_len",
                  "storage_count", "gas_min", "gas_max", "gas_limit"):
            getattr(b, f)[i] = getattr(c2, f)[i]
        b.calldata[i] = c2.calldata[i]
        b.env[i] = c2.env[i]
        b.storage[i] = c2.storage[i, :16]
    for k in range(2 * len(CRAFTED)):
        i = n_c2 + k
        b.set_lane(i, calldata=b"", address=workloads.CONTRACT, caller=0xDEADBEEF + k, origin=k % 2,
                   callvalue=3, gasprice=1, gas_limit=2000 if k // 2 == len(CRAFTED) - 1 else 8_000_000)
    b.flags[:] |= MG_LANE_TAINT
    b.n_obj[:] = MG_TAINT_OBJ0
    b.n_fixed[:] = MG_TAINT_OBJ0
    b.tflags[::5] = 2                 # these lanes' states carry the if-annotation class
    return b, codes, n_c2


def _load(dev, b, codes, n_c2):
    ids = [dev.load_code(c) for c in codes]
    b.code_id[:n_c2] = ids[0]
    for k in range(2 * len(CRAFTED)):
        b.code_id[n_c2 + k] = ids[1 + k // 2]


def _partition(b, i):
    """Per stack slot: (object class, atoms) with classes numbered by first
    appearance; handle-0 slots are objects of their own."""
    seen, out = {}, []
    for s in range(int(b.sp[i])):
        h = int(b.sobj[i, s])
        key = ("fresh", s) if h == 0 else h
        if key not in seen:
            seen[key] = len(seen)
        out.append((seen[key], int(b.omask[i, h]) if h else 0))
    env = [int(b.omask[i, h]) for h in range(1, 7)]
    return out, env


@pytest.mark.parametrize("obj_cap", [64, 16])
def test_device_taint_planes_match_the_restatement(obj_cap):
    hook = [0, 0, 0, 0]
    for op in ("STOP", "RETURN"):
        o = OPCODES[op]
        hook[o >> 6] |= 1 << (o & 63)
    b, codes, n_c2 = _batch(obj_cap=obj_cap)
    gpu = GpuDevice(0)
    try:
        _load(gpu, b, codes, n_c2)
        ref = b.copy()
        ora = OracleDevice()
        for c in codes:
            ora.load_code(c)
        gpu.alloc(b.shape)
        gpu.set_taint_program(ACTIONS)
        gpu.upload(b)
        ora.alloc(b.shape)
        ora.set_taint_program(ACTIONS)
        ora.upload(ref)
        for _ in range(3):          # yields and budget pauses resume like the host would
            st = gpu.step(hook, max_steps=400)
            ora.step(hook, max_steps=400)
        gpu.download(b)
        ora.download(ref)
    finally:
        gpu.close()
    assert st.lane_steps >= 0
    for f in ("pc", "sp", "status", "aux", "steps", "gas_min", "gas_max", "rec_len", "n_atoms", "sink",
              "ymask", "tflags"):
        assert np.array_equal(getattr(b, f), getattr(ref, f)), f
    for i in range(b.n):
        assert np.array_equal(b.rec[i, : int(b.rec_len[i])], ref.rec[i, : int(ref.rec_len[i])]), i
        assert _partition(b, i) == _partition(ref, i), i
        assert np.array_equal(b.stack[i, : int(b.sp[i])], ref.stack[i, : int(ref.sp[i])]), i
    # the crafted cases happened
    k0 = n_c2
    assert int(b.status[k0 + 2]) == 7                         # ORIGIN == 0 at the JUMPI: yield
    assert int(b.aux[k0 + 12]) >> 8 == 9                      # 64 atoms: MG_ESC_TAINT
    assert int(b.status[k0 + 14]) == 6                        # the DUP loop runs out of gas
    assert (b.tflags[:n_c2] & 1).any() and b.n_atoms[:n_c2].max() > 0


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
@pytest.mark.parametrize("modules", ["integer+origin", "default"])
def test_laser_taint_on_the_gpu_matches_host_hooks(strategy, modules, monkeypatch):
    import test_taint_cpu as t
    mods = t.DEFAULT_SET if modules == "default" else ("IntegerArithmetics", "TxOrigin")
    gpu = GpuDevice(0)
    try:
        ends_d, issues_d, launches_d, steps_d = t._run(strategy, "device", monkeypatch, device=gpu, modules=mods)
        ends_h, issues_h, launches_h, steps_h = t._run(strategy, "host", monkeypatch, device=gpu, modules=mods)
        ends_c, issues_c, _, steps_c = t._run(strategy, "device", monkeypatch, modules=mods)   # oracle device
    finally:
        gpu.close()
    assert steps_d == steps_h == steps_c
    assert ends_d == ends_h == ends_c
    assert issues_d == issues_h == issues_c
    assert launches_d < launches_h
