"""Host layer of the batched LASER core (mythril_amd/laser) — CPU tests.

These check the parts that do not step paths: the opcode table against the
reference's (golden fixture), the host disassembly against the oracle's, the hook
registration API and its error behaviour (svm.py:639-782), state objects, and the
event-order rules of LaserEVM.exec.  Device stepping through LaserEVM is covered
by tests/test_gpu_laser.py.
"""
import json

import numpy as np
import pytest

from mythril_amd.lanes import (LaneBatch, LaneShape, MG_HALT_STOP, MG_HOOK, MG_VMEXC)
from mythril_amd.laser import (Account, Disassembly, LaserEVM, MachineStack, WorldState,
                               execute_message_call)
from mythril_amd.laser import opcodes
from mythril_amd.laser.state import StackUnderflowException
from mythril_amd.laser.svm import _event_round, _next_event, _Lane, _ranges
from vmtests_util import GOLDEN, load_vmtests


def test_opcode_table_matches_reference():
    ref = json.loads((GOLDEN / "opcodes.json").read_text())
    assert set(ref) == set(opcodes.OPCODES)
    for name, rec in ref.items():
        assert opcodes.OPCODES[name] == rec["byte"]
        assert opcodes.get_required_stack_elements(name) == rec["stack"][0], name
        assert tuple(opcodes.get_opcode_gas(name)) == tuple(rec["gas"]), name


def _codes():
    codes = [bytes.fromhex(h) for h in json.loads((GOLDEN / "bytecodes.json").read_text()).values()]
    codes += list({bytes.fromhex(v["code"]) for v in load_vmtests()})
    # truncated PUSH at the end, unknown bytes, PUSH0, bzzr tail
    codes += [bytes.fromhex("6001600261"), bytes.fromhex("5f0c0d21fe"),
              b"\x60\x01" + b"\x00" * 8 + b"bzzr0" + b"\x11" * 38]
    return codes


def test_disassembly_matches_oracle_tables(oracle_evm):
    o = oracle_evm()
    for code in _codes():
        cid = o.load_code(code)
        ops, addrs = o.code_table(cid)
        ins = Disassembly(code).instruction_list
        assert [i["address"] for i in ins] == addrs.tolist()
        assert [opcodes.OPCODES.get(i["opcode"], 0xFE) if i["opcode"] != "INVALID" else 0xFE
                for i in ins] == [b if b in opcodes.ADDRESS_OPCODE_MAPPING else 0xFE
                                  for b in ops.tolist()]


def test_disassembly_push_argument_and_hex_input():
    d = Disassembly("0x6001610203")
    assert d.instruction_list == [
        {"address": 0, "opcode": "PUSH1", "argument": "0x01"},
        {"address": 2, "opcode": "PUSH2", "argument": "0x0203"}]
    assert Disassembly("61ff").instruction_list == [
        {"address": 0, "opcode": "PUSH2", "argument": "0xff"}]


def test_hook_registration_api():
    vm = LaserEVM(requires_statespace=False, device=object())
    seen = []
    vm.register_hooks("pre", {"SSTORE": [lambda s: seen.append("a")]})
    vm.register_hooks("post", {"SLOAD": [lambda s: seen.append("b")]})
    with pytest.raises(ValueError):
        vm.register_hooks("middle", {})
    with pytest.raises(ValueError):
        vm.register_laser_hooks("no_such_hook", lambda: None)

    @vm.laser_hook("add_world_state")
    def h(state):
        pass
    assert vm._add_world_state_hooks == [h]

    @vm.pre_hook("ADD")
    def p(state):
        pass

    @vm.post_hook("ADD")
    def q(state):
        pass
    assert vm.pre_hooks["ADD"] == [p] and vm.post_hooks["ADD"] == [q]

    # opcode None: a factory called once per opcode (svm.py:658-667)
    made = []
    vm.instr_hook("pre", None)(lambda op: made.append(op) or (lambda s: None))
    assert sorted(made) == sorted(opcodes.OPCODES)
    hooked = vm._hooked_ops()
    assert hooked == set(range(256)) - (set(range(256)) - set(opcodes.ADDRESS_OPCODE_MAPPING))


def test_hooked_ops_and_post_detection():
    vm = LaserEVM(requires_statespace=False, device=object())
    assert vm._hooked_ops() == set()
    vm.register_hooks("pre", {"SSTORE": [lambda s: None]})
    vm.register_instr_hooks("post", "JUMPI", lambda s: None)
    assert vm._hooked_ops() == {0x55, 0x57}
    assert not vm._has_post("SSTORE") and vm._has_post("JUMPI")
    vm.register_laser_hooks("execute_state", lambda s: None)
    assert vm._hooked_ops() == set(range(256))


def test_lane_shape_is_a_valid_batch_configuration():
    vm = LaserEVM(requires_statespace=False, device=object())
    ws = WorldState()
    ws.put_account(Account(1, code=Disassembly("00")))
    vm.open_states = [ws]
    captured = {}
    vm.exec = lambda track_gas=False: captured.setdefault("work", list(vm.work_list))
    execute_message_call(vm, 1, 2, 2, data=b"\x01" * 37, gas_limit=10, gas_price=0, value=0)
    shape = vm._shape(captured["work"])
    assert shape.mem_cap % 32 == 0 and shape.calldata_cap % 4 == 0 and shape.calldata_cap >= 37
    assert 0 < shape.stack_cap <= 1024 and shape.storage_cap > 0


def test_machine_stack_semantics():
    st = MachineStack()
    with pytest.raises(StackUnderflowException):
        st.pop()
    st.append(5)
    assert st[-1].value == 5
    with pytest.raises(StackUnderflowException):
        st[-2]


def test_execute_message_call_builds_states():
    vm = LaserEVM(requires_statespace=False, device=object())
    ws = WorldState()
    acct = Account(0x1234, code=Disassembly("6001600055"))
    acct.storage[7] = 9
    ws.put_account(acct)
    vm.open_states = [ws]
    captured = {}
    vm.exec = lambda track_gas=False: captured.setdefault("work", list(vm.work_list))
    execute_message_call(vm, callee_address=0x1234, caller_address=0xCAFE, origin_address=0xCAFE,
                         code="6001600055", gas_limit=100000, data=b"\x01\x02", gas_price=1, value=0,
                         track_gas=True)
    (s,) = captured["work"]
    assert vm.open_states == []
    assert s.environment.calldata == b"\x01\x02"
    assert s.environment.active_account.storage[7].value == 9
    assert s.current_transaction.gas_limit == 100000
    assert s.get_current_instruction() == {"address": 0, "opcode": "PUSH1", "argument": "0x01"}


def _fake_batch(rows):
    """rows: (status, steps) per lane."""
    b = LaneBatch(LaneShape(n=len(rows), stack_cap=1, mem_cap=32, calldata_cap=4, storage_cap=1))
    for i, (st, steps) in enumerate(rows):
        b.status[i], b.steps[i] = st, steps
    return b


def test_event_order_bfs_and_dfs():
    # lane 0 halts executing its 5th instruction (round 4), lane 1 hooks before
    # its 4th (round 3), lane 2 throws in its 4th (round 3)
    b = _fake_batch([(MG_HALT_STOP, 5), (MG_HOOK, 3), (MG_VMEXC, 4)])
    assert [_event_round(b, i) for i in range(3)] == [4, 3, 3]
    lanes = [_Lane(None, i) for i in range(3)]
    for ln in lanes:
        ln.phase = "event"
    order_bfs, order_dfs = [], []
    for order, bfs in ((order_bfs, True), (order_dfs, False)):
        for ln in lanes:
            ln.phase = "event"
        while True:
            e = _next_event(lanes, b, bfs)
            if e is None:
                break
            order.append(e)
            lanes[e].phase = "done"
    assert order_bfs == [1, 2, 0]
    assert order_dfs == [2, 1, 0]
    assert _ranges([5, 1, 2, 3, 9]) == [[1, 3], [5, 1], [9, 1]]


def test_statespace_graph_is_empty_without_the_flag():
    """Without requires_statespace the lanes run free and no graph is kept
    (the reference does not create the attributes at all, svm.py:94-97); the
    graph itself is tested in test_statespace_cpu.py."""
    from mythril_amd.laser import LaserEVM
    from oracle_device import OracleDevice
    vm = LaserEVM(device=OracleDevice(), requires_statespace=False)
    assert vm.nodes == {} and vm.edges == []
