"""The dispatcher's function table and active_function_name on CPU.

* Disassembly.get_easm() against the reference's own expected outputs
  (tests/testdata/outputs_expected/*.easm, disassembler_test.py:13-27; as data in
  tests/golden/easm.json), from the host disassembly and from the oracle's code
  table.  Two files use opcode names the reference's table has since renamed
  (0xff SUICIDE -> SELFDESTRUCT, 0xfe ASSERT_FAIL -> INVALID:
  support/opcodes.py:130 and :131); overflow.sol.o.easm disassembles another
  compilation than tests/testdata/inputs/overflow.sol.o (its first PUSH is 0x60,
  the input's 0x80).  The reference's own test never compares them: it skips a
  file unless an output of the current run already exists
  (disassembler_test.py:17-19).
* The table itself (disassembly.py:36-114): function hashes and entry points,
  names from a signature database or ``_function_0x<hash>``; the host's entry set
  equals the oracle's independent restatement on every reference bytecode.
* The per-lane record of the last function-entry landing (mg_lane_soa.fent) on
  the C oracle equals a single-step restatement of the reference's exec loop
  (svm.py:293-337 + manage_cfg), and LaserEVM maps it to the same names.
"""
import json

import numpy as np
import pytest

from fnames import GOLDEN, easm_from_table, names_by_single_step, selector, use_signature_db
from mythril_amd import workloads
from mythril_amd.lanes import MG_FENT_NONE, LaneBatch, LaneShape
from mythril_amd.laser.disassembly import Disassembly, SignatureDB

EASM = json.loads((GOLDEN / "easm.json").read_text())
BYTECODES = json.loads((GOLDEN / "bytecodes.json").read_text())
RENAMED = {" SUICIDE\n": " SELFDESTRUCT\n", " ASSERT_FAIL\n": " INVALID\n"}
STALE = {"overflow.sol.o"}


def _expected(name: str) -> str:
    text = EASM[name]
    for old, new in RENAMED.items():
        text = text.replace(old, new)
    return text


@pytest.fixture(autouse=True)
def _no_user_db(monkeypatch, tmp_path):
    monkeypatch.setenv("MYTHRIL_DIR", str(tmp_path / "empty"))
    SignatureDB._reset()
    yield
    SignatureDB._reset()


def test_easm_goldens_on_the_host_and_the_oracle_table():
    from oracle.evm_ref import OracleEVM
    o = OracleEVM()
    exact = renamed = 0
    for name, text in sorted(EASM.items()):
        code = BYTECODES[name]
        host = Disassembly(code).get_easm()
        raw = bytes.fromhex(code[2:] if code.startswith("0x") else code)
        ops, addrs = o.code_table(o.load_code(raw))
        assert easm_from_table(ops, addrs, raw) == host, name
        if name in STALE:
            assert text.splitlines()[0] == "0 PUSH1 0x60" and host.splitlines()[0] == "0 PUSH1 0x80"
            continue
        assert host == _expected(name), name
        exact += host == text
        renamed += host != text
    assert (exact, renamed) == (10, 2)


def test_function_table_names_and_hashes():
    d = Disassembly(BYTECODES["overflow.sol.o"])
    assert d.func_hashes == ["0x18160ddd", "0x70a08231", "0xa3210e87"]
    assert d.address_to_function_name == {92: "_function_0x18160ddd", 135: "_function_0x70a08231",
                                          236: "_function_0xa3210e87"}
    assert d.function_name_to_address == {v: k for k, v in d.address_to_function_name.items()}
    # PUSH1 / PUSH2 hashes are left-padded to 8 digits (disassembly.py:97)
    d2 = Disassembly("60aa1461000a5760025b00")
    assert d2.func_hashes == ["0x000000aa"] and d2.address_to_function_name == {10: "_function_0x000000aa"}


def test_signature_database_names(monkeypatch, tmp_path):
    use_signature_db(monkeypatch, tmp_path)
    d = Disassembly(BYTECODES["ether_send.sol.o"])
    assert sorted(d.address_to_function_name.values()) == sorted(json.loads(
        (GOLDEN / "signatures.json").read_text())["ether_send.sol"])
    assert SignatureDB().get(selector("kill(address)")) == ["kill(address)"]


def test_host_entry_set_equals_the_oracle_restatement():
    from oracle.evm_ref import OracleEVM
    o = OracleEVM()
    codes = dict(BYTECODES)
    codes["disassembly.json"] = json.loads((GOLDEN / "disassembly.json").read_text())["code"]
    # a dispatcher whose entry is the JUMPI's fall-through, a PUSH4 entry, an
    # entry past the end of the code, and one cut off by the end of the code
    codes["synthetic"] = "6001146007575b00" + "63aabbccdd14600d575b" + "6001146101005700" + "60021461"
    n_entries = 0
    for name, code in codes.items():
        raw = bytes.fromhex(code[2:] if code.startswith("0x") else code)
        host = np.array(Disassembly(code).function_entries(), dtype=np.uint8)
        dev = o.code_fentries(o.load_code(raw))
        assert np.array_equal(host, dev), name
        n_entries += int(host.sum())
    assert n_entries > 60


def _c2_lanes(n):
    code = workloads.bytecode("overflow.sol.o")
    from oracle.evm_ref import OracleEVM
    o = OracleEVM()
    cid = o.load_code(code)
    b = workloads.c2_batch(n, code_id=cid, stack_cap=64, mem_cap=1024)
    return o, b, code


def test_lane_function_entry_record_equals_single_step_restatement():
    o, b, code = _c2_lanes(96)
    d = Disassembly(code)
    ref = b.copy()
    o.run(b)
    names = {}
    for i in range(b.n):
        want = names_by_single_step(o, ref, i, d)
        fe = int(b.fent[i])
        got = "fallback" if fe == MG_FENT_NONE else (d.name_at(fe) or "fallback")
        assert got == want, (i, fe, want)
        names[want] = names.get(want, 0) + 1
    # the three dispatcher functions and the fall-through all occur
    assert set(names) == {"_function_0x18160ddd", "_function_0x70a08231", "_function_0xa3210e87", "fallback"}


def test_laser_function_names_batched_equal_single_step(monkeypatch, tmp_path):
    """LaserEVM on the oracle device: the name every path ends with (a
    transaction_end hook records it) for concrete calls into overflow.sol.o, one
    per selector and a fall-through, equals the single-step restatement's."""
    use_signature_db(monkeypatch, tmp_path)
    from oracle_device import OracleDevice
    from mythril_amd.laser import Account, LaserEVM, WorldState
    from mythril_amd.laser.transaction import execute_message_call
    code = workloads.bytecode("overflow.sol.o")
    calls = [bytes.fromhex(selector("totalSupply()")[2:]),
             bytes.fromhex(selector("balanceOf(address)")[2:]) + (7).to_bytes(32, "big"),
             bytes.fromhex(selector("sendeth(address,uint256)")[2:]) + (7).to_bytes(32, "big") + (0).to_bytes(32, "big"),
             b"\x01\x02\x03\x04"]
    seen = []
    for data in calls:
        vm = LaserEVM(device=OracleDevice(), requires_statespace=False)
        vm.register_laser_hooks("transaction_end",
                                lambda st, tx, ret, rev: seen.append(st.environment.active_function_name))
        ws = WorldState()
        acct = Account(0x1234, code=Disassembly(code), contract_name="MAIN")
        ws.put_account(acct)
        vm.open_states = [ws]
        execute_message_call(vm, callee_address=0x1234, caller_address=0xDEADBEEF, origin_address=0xDEADBEEF,
                             data=data, gas_limit=8_000_000, gas_price=1, value=0)
    assert seen == ["totalSupply()", "balanceOf(address)", "sendeth(address,uint256)", "fallback"]
