"""Reference state tests (tests/laser/state/*_test.py, via tests/golden/
state_cases.json) against the host mirror and, as lane programs, against the C
oracle; tests/test_gpu_state_pins.py runs the same programs on kernel 1."""
import random

import pytest

import state_pins
from mythril_amd.laser.state import (MachineStack, MachineState, Memory, StackOverflowException,
                                     StackUnderflowException, Storage)
from mythril_amd.laser.symbolic import SymbolicCalldata
from mythril_amd.laser.witness import eval_all
from mythril_amd.smt.expr import Expression, symbol_factory
from mythril_amd.smt.program import ArrayInterp
from oracle_device import OracleDevice

C = state_pins.CASES
BVV = symbol_factory.BitVecVal


def test_lane_programs_on_the_oracle():
    state_pins.check(state_pins.run_programs(OracleDevice()))


# ---- calldata_test.py ----------------------------------------------------------------
def _random_models(names, n=64, seed=0, fixed=None):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        a = {k: rng.getrandbits(256) for k in names}
        a["0_calldata"] = ArrayInterp(rng.getrandbits(8), {rng.randrange(64): rng.getrandbits(8) for _ in range(8)})
        a.update(fixed or {})
        out.append(a)
    return out


def test_symbolic_calldata_index_past_size_is_zero():
    """calldata_test.py:58-73: calldata[51] == 1 and calldatasize == 50 is unsat:
    the byte is If(51 < size, ...) -> 0 under every model with size 50."""
    case = C["calldata"]["symbolic_index"]
    cd = SymbolicCalldata("0")
    v = cd[case["index"]]
    vals = eval_all(v.raw, _random_models([], fixed={"0_calldatasize": case["size"]}))
    assert all(x != case["value"] for x in vals) and not case["sat"]
    # and inside the size the byte is the array's (a model exists)
    vals = eval_all(v.raw, _random_models([], fixed={"0_calldatasize": case["index"] + 1}))
    assert any(x != 0 for x in vals)


def test_symbolic_calldata_equal_indices_give_equal_bytes():
    """calldata_test.py:76-91: index_a == index_b and calldata[a] != calldata[b] is unsat."""
    cd = SymbolicCalldata("0")
    ia, ib = symbol_factory.BitVecSym("index_a", 256), symbol_factory.BitVecSym("index_b", 256)
    ne = cd[ia] != cd[ib]
    rng = random.Random(1)
    models = []
    for _ in range(64):
        k = rng.randrange(64)
        models.append({"index_a": k, "index_b": k, "0_calldatasize": rng.randrange(128),
                       "0_calldata": ArrayInterp(0, {j: rng.getrandbits(8) for j in range(64)})})
    assert not any(eval_all(ne.raw, models)) and not C["calldata"]["symbolic_equal_indices"]["sat"]


# ---- storage_test.py -------------------------------------------------------------------
@pytest.mark.parametrize("init,key", C["storage"]["uninitialized"])
def test_storage_uninitialized_index(init, key):
    concrete = Storage(concrete=True)
    symbolic = Storage(concrete=False, address=0x1234)
    for k, v in init.items():
        concrete[BVV(int(k), 256)] = BVV(v, 256)
        symbolic[BVV(int(k), 256)] = BVV(v, 256)
    assert concrete[BVV(key, 256)].value == 0
    got = symbolic[BVV(key, 256)]
    assert isinstance(got, Expression) and got.symbolic


def test_storage_set_and_change_item():
    si, ci = C["storage"]["set_item"], C["storage"]["change_item"]
    s = Storage()
    s[BVV(si["key"], 256)] = BVV(si["value"], 256)
    assert s[BVV(si["key"], 256)].value == si["value"]
    s = Storage()
    for v in ci["values"]:
        s[BVV(ci["key"], 256)] = BVV(v, 256)
    assert s[BVV(ci["key"], 256)].value == ci["expected"]


# ---- mstate_test.py / mstack_test.py ----------------------------------------------------
@pytest.mark.parametrize("initial,start,ext", C["mstate"]["memory_extension"])
def test_memory_extension(initial, start, ext):
    ms = MachineState(gas_limit=8_000_000)
    ms.memory = Memory()
    ms.memory.extend(initial)
    ms.mem_extend(start, ext)
    assert ms.memory_size == len(ms.memory) == max(initial, (start + ext + 31) // 32 * 32)


@pytest.mark.parametrize("size,over", C["mstate"]["stack_pop_too_many"])
def test_stack_pop_too_many(size, over):
    ms = MachineState(8_000_000)
    ms.stack = MachineStack([42] * size)
    with pytest.raises(StackUnderflowException):
        ms.pop(size + over)


@pytest.mark.parametrize("stack,amount,expected", C["mstate"]["stack_pop"])
def test_stack_multiple_pop(stack, amount, expected):
    ms = MachineState(8_000_000)
    ms.stack = MachineStack(stack[:])
    got = ms.pop(amount)
    assert list(got) == stack[-amount:][::-1] == expected
    assert len(ms.stack) == len(stack) - amount


def test_memory_zeroed_and_write():
    z, w = C["mstate"]["memory_zeroed"], C["mstate"]["memory_write"]
    mem = Memory()
    mem.extend(z["extend"])
    mem[z["byte"][0]] = z["byte"][1]
    mem.write_word_at(z["word"][0], z["word"][1])
    assert all(mem[k] == 0 for k in z["zero_bytes"]) and mem.get_word_at(z["zero_word"]).value == 0
    mem = Memory()
    mem.extend(w["extend"])
    a = symbol_factory.BitVecSym("a", 256)
    b = symbol_factory.BitVecSym("b", 8)
    mem[w["byte"][0]] = w["byte"][1]
    mem[w["sym_byte"]] = b
    mem.write_word_at(w["word"][0], w["word"][1])
    mem.write_word_at(w["sym_word"], a)
    for k, v in w["expect_byte"]:
        assert mem[k] == v
    assert mem.get_word_at(w["word"][0]).value == w["word"][1]
    assert mem.get_word_at(w["sym_word"]).raw is a.raw          # simplify(a == word) is True
    assert mem[w["sym_byte"]].raw is b.raw


def test_machine_stack():
    mc = C["mstack"]
    assert MachineStack(mc["constructor"]) == mc["constructor"]
    st = MachineStack()
    for _ in range(mc["limit"]):
        st.append(1)
    with pytest.raises(StackOverflowException):
        st.append(1000)
    st = MachineStack(mc["pop"]["stack"])
    assert st.pop() == mc["pop"]["value"]
    with pytest.raises(StackUnderflowException):
        st.pop()
    with pytest.raises(NotImplementedError):
        MachineStack([0, 1]) + [2]
    with pytest.raises(NotImplementedError):
        st = MachineStack()
        st += st


@pytest.mark.parametrize("name,code", state_pins.symbolic_programs())
def test_symbolic_fixture_programs_on_the_restatement(name, code):
    """The same symbolic programs through the CPU restatement (tests/symref.py),
    the oracle the GPU test compares kernel 1 with."""
    import symref
    s, eng = state_pins.symbolic_state(code), symref.Engine()
    while True:
        out = eng.step(s)
        if not out:
            break
        s = out[0]
    kind, last = eng.ended[-1]
    assert kind == "stop"
    state_pins.check_symbolic_stack(name, last.mstate.stack)
