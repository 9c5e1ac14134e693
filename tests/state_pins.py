"""The reference's state tests (tests/laser/state/{calldata,storage,mstate,
mstack}_test.py, as data in tests/golden/state_cases.json) restated twice:

* on the host mirror (mythril_amd/laser/state.py, symbolic.py) exactly as the
  reference tests drive their classes -- test_state_pins_cpu.py;
* as EVM programs on lanes (calldata reads, storage reads/writes, memory
  extension, stack pops), whose results land in storage slots, run on any
  device with the GpuDevice interface: the C oracle (CPU suite) and kernel 1
  (tests/test_gpu_state_pins.py).  A case whose state the EVM cannot reach is
  pinned on the host only (an initial memory of 100 bytes: execution grows
  memory in 32-byte words, machine_state.py:143).
"""
from __future__ import annotations

import json
from pathlib import Path

from mythril_amd.lanes import LaneBatch, LaneShape, MG_EXC_STACK_UNDERFLOW, MG_VMEXC, WORLD_STATE_KEPT

CASES = json.loads((Path(__file__).resolve().parent / "golden" / "state_cases.json").read_text())


def push(v: int) -> bytes:
    n = max(1, (v.bit_length() + 7) // 8)
    return bytes([0x5F + n]) + v.to_bytes(n, "big")


CALLDATALOAD, CALLDATASIZE, CALLDATACOPY = b"\x35", b"\x36", b"\x37"
SLOAD, SSTORE, MLOAD, MSTORE, MSTORE8, MSIZE = b"\x54", b"\x55", b"\x51", b"\x52", b"\x53", b"\x59"
SHR, POP, STOP = b"\x1c", b"\x50", b"\x00"


def store_top(slot: int) -> bytes:
    return push(slot) + SSTORE


def byte_at_top() -> bytes:                  # the top word's most significant byte
    return push(248) + SHR


def programs():
    """[(name, code, calldata, initial storage, expect)] where expect is
    {slot: value} (an open world state) or "exception"."""
    out = []
    c = CASES["calldata"]
    rd = c["uninitialized_reads"]
    for data in c["uninitialized"] + [c["calldatasize"]["data"]]:
        idx = c["constrain_index"]["index"]
        code = (push(rd["index"]) + CALLDATALOAD + byte_at_top() + store_top(0x10) +
                push(rd["word_at"]) + CALLDATALOAD + store_top(0x11) +
                CALLDATASIZE + store_top(0x12) +
                push(idx) + CALLDATALOAD + byte_at_top() + store_top(0x13) + STOP)
        exp = {0x10: rd["expected"], 0x11: rd["expected"], 0x12: len(data),
               0x13: data[idx] if idx < len(data) else 0}
        out.append((f"calldata{len(data)}", code, bytes(data), {}, exp))
    s = CASES["storage"]
    si, ci = s["set_item"], s["change_item"]
    for init, key in s["uninitialized"]:
        init = {int(k): v for k, v in init.items()}
        code = (push(key) + SLOAD + store_top(0x20) +
                push(si["value"]) + push(si["key"]) + SSTORE + push(si["key"]) + SLOAD + store_top(0x21))
        for v in ci["values"]:
            code += push(v) + push(ci["key"]) + SSTORE
        code += push(ci["key"]) + SLOAD + store_top(0x22) + STOP
        out.append((f"storage{len(init)}_{key}", code, b"", init,
                    {0x20: 0, 0x21: si["value"], 0x22: ci["expected"]}))
    m = CASES["mstate"]
    for init, start, ext in m["memory_extension"]:
        if init % 32:
            continue                      # host only (module docstring)
        code = b""
        if init:
            code += push(0) + push(init - 1) + MSTORE8
        code += push(ext) + push(0) + push(start) + CALLDATACOPY + MSIZE + store_top(0x30) + STOP
        out.append((f"memext{init}_{start}_{ext}", code, b"", {},
                    {0x30: max(init, (start + ext + 31) // 32 * 32)}))
    for n, over in m["stack_pop_too_many"]:
        code = push(42) * n + POP * (n + over) + STOP
        out.append((f"underflow{n}_{over}", code, b"", {}, "exception"))
    for stack, amount, expected in m["stack_pop"]:
        code = b"".join(push(v) for v in stack)
        for j in range(amount):              # SSTORE pops the slot, then the popped value
            code += store_top(0x40 + j)
        out.append((f"pop{len(stack)}_{amount}", code + STOP, b"", {},
                    {0x40 + j: v for j, v in enumerate(expected)}))
    z, w = m["memory_zeroed"], m["memory_write"]
    code = (push(z["byte"][1]) + push(z["byte"][0]) + MSTORE8 + push(z["word"][1]) + push(z["word"][0]) + MSTORE)
    for j, k in enumerate(z["zero_bytes"]):
        code += push(k) + MLOAD + byte_at_top() + store_top(0x50 + j)
    code += push(z["zero_word"]) + MLOAD + store_top(0x52) + STOP
    out.append(("memory_zeroed", code, b"", {}, {0x50: 0, 0x51: 0, 0x52: 0}))
    code = (push(w["byte"][1]) + push(w["byte"][0]) + MSTORE8 + push(w["word"][1]) + push(w["word"][0]) + MSTORE)
    exp = {}
    for j, (k, v) in enumerate(w["expect_byte"]):
        code += push(k) + MLOAD + byte_at_top() + store_top(0x60 + j)
        exp[0x60 + j] = v
    code += push(w["word"][0]) + MLOAD + store_top(0x68) + STOP
    exp[0x68] = w["word"][1]
    out.append(("memory_write", code, b"", {}, exp))
    return out


def run_programs(dev):
    """Run every program on `dev`; return [(name, status, storage dict, expect)]."""
    progs = programs()
    shape = LaneShape(n=len(progs), stack_cap=1024, mem_cap=4096, calldata_cap=64, storage_cap=32)
    b = LaneBatch(shape)
    for i, (name, code, data, init, _) in enumerate(progs):
        b.set_lane(i, code_id=dev.load_code(code), calldata=data, address=0x1234, storage=init)
    dev.alloc(shape)
    dev.upload(b)
    dev.step()
    out = LaneBatch(shape)
    dev.download(out)
    return [(name, (int(out.status[i]), int(out.aux[i])), out.storage_dict(i, drop_zero=False), exp)
            for i, (name, _, _, _, exp) in enumerate(progs)]


def check(results):
    for name, status, storage, exp in results:
        if exp == "exception":         # StackUnderflowException (machine_state.py:58-71)
            assert status == (MG_VMEXC, MG_EXC_STACK_UNDERFLOW), (name, status)
            continue
        assert status[0] in WORLD_STATE_KEPT, (name, status)
        got = {k: storage.get(k, 0) for k in exp}
        assert got == exp, (name, got, exp)


# ---- symbolic lanes: the fixture's symbolic cases as programs ------------------------------
def symbolic_programs():
    """[(name, code)] run on a symbolic lane (symbolic calldata, storage): the
    calldata byte at the fixture's index past its size (calldata_test.py:58-73),
    two loads at the same symbolic index (:76-91), and an uninitialised read of
    symbolic storage after the fixture's stores (storage_test.py:27-38)."""
    c, st = CASES["calldata"]["symbolic_index"], CASES["storage"]["uninitialized"]
    out = [("cd_index", push(c["index"]) + CALLDATALOAD + byte_at_top() + STOP),
           # index_a == index_b: the index is one calldata word loaded twice
           ("cd_equal", push(0) + CALLDATALOAD + CALLDATALOAD + push(0) + CALLDATALOAD + CALLDATALOAD + STOP)]
    for init, key in st:
        code = b"".join(push(v) + push(int(k)) + SSTORE for k, v in init.items())
        out.append((f"sym_storage{len(init)}_{key}", code + push(key) + SLOAD + STOP))
    return out


def symbolic_state(code: bytes, txid: str = "7"):
    """A symbolic message call's initial state into `code`, with symbolic storage."""
    from mythril_amd import workloads
    from mythril_amd.laser import Account, Disassembly, MessageCallTransaction, SymbolicCalldata, WorldState
    from mythril_amd.smt.expr import symbol_factory
    ws = WorldState()
    acct = Account(workloads.CONTRACT, code=Disassembly(code), concrete_storage=False)
    ws.put_account(acct)
    sender = symbol_factory.BitVecSym(f"sender_{txid}", 256)
    tx = MessageCallTransaction(world_state=ws, identifier=txid, gas_limit=8_000_000, origin=sender,
                                caller=sender, callee_account=acct, call_data=SymbolicCalldata(txid),
                                call_value=symbol_factory.BitVecSym(f"call_value{txid}", 256),
                                gas_price=symbol_factory.BitVecSym(f"gas_price{txid}", 256))
    gs = tx.initial_global_state()
    gs.transaction_stack.append((tx, None))
    return gs


def check_symbolic_stack(name: str, stack, txid: str = "7"):
    """The reference tests' verdicts on the final stack of a symbolic program."""
    import random
    from mythril_amd.laser.witness import eval_all
    from mythril_amd.smt.expr import Expression
    from mythril_amd.smt.program import ArrayInterp
    rng = random.Random(5)
    if name == "cd_index":
        c = CASES["calldata"]["symbolic_index"]
        models = [{f"{txid}_calldatasize": c["size"],
                   f"{txid}_calldata": ArrayInterp(rng.getrandbits(8), {c["index"]: rng.getrandbits(8)})}
                  for _ in range(32)]
        assert all(v != c["value"] for v in eval_all(stack[-1].raw, models)) and not c["sat"]
    elif name == "cd_equal":
        assert stack[-1].raw is stack[-2].raw                 # the same term: a != b is unsat
    else:
        got = stack[-1]
        assert isinstance(got, Expression) and got.symbolic   # storage_test.py:27-38
