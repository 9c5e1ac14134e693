"""Pin the CPU oracle (oracle/evm_ref.c) before trusting it as the GPU checker.

Sources of truth, all data from the reference's own tests (tests/golden/):
  * VMTests post-states, judged as tests/laser/evm_testsuite/evm_test.py:153-189;
  * EIP-145 SHL/SHR/SAR vectors (tests/instructions/{shl,shr,sar}_test.py);
  * keccak256("") (keccak_function_manager.py:92);
  * the opcode gas/stack table (support/opcodes.py:16-144);
plus random operands against the pure-Python restatement in tests/pysem.py.
"""
import hashlib
import random

import numpy as np
import pytest

import pysem
from mythril_amd.lanes import (LaneBatch, LaneShape, MG_HALT_STOP, MG_VMEXC, MG_ESCAPE,
                               MG_EXC_STACK_UNDERFLOW, limbs_to_word)
from oracle.evm_ref import OracleEVM, keccak256, opcode_info
from vmtests_util import fill_lane, judge, load_json, load_vmtests, vm_shape

# vectors the oracle hands to the host (symbolic or world-state opcodes): NUMBER,
# BLOCKHASH, SELFDESTRUCT, and a SHA3 whose memory outgrows a 1 MiB lane page.
EXPECTED_ESCAPES = {
    "BlockNumberDynamicJump0_AfterJumpdest", "BlockNumberDynamicJump0_AfterJumpdest3",
    "BlockNumberDynamicJump0_withoutJumpdest", "BlockNumberDynamicJump1",
    "BlockNumberDynamicJumpInsidePushWithJumpDest",
    "BlockNumberDynamicJumpInsidePushWithoutJumpDest", "DynamicJumpJD_DependsOnJumps0",
    "DynamicJumpPathologicalTest1", "DynamicJumpPathologicalTest2",
    "DynamicJumpPathologicalTest3", "201503102320PYTHON", "201503110206PYTHON",
    "201503110219PYTHON", "201503112218PYTHON", "push32AndSuicide", "suicide0",
    "suicideNotExistingAccount", "suicideSendEtherToMe", "suicide", "sha3_bigOffset2",
}


def run_vmtests(vectors):
    o = OracleEVM()
    b = LaneBatch(vm_shape(vectors))
    codes = {}
    for i, v in enumerate(vectors):
        if v["code"] not in codes:
            codes[v["code"]] = o.load_code(bytes.fromhex(v["code"]))
        fill_lane(b, i, v, codes[v["code"]])
    o.run(b)
    return b


def test_vmtests_post_states():
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    assert len(vectors) == 519
    b = run_vmtests(vectors)
    fails, escaped = [], set()
    for i, v in enumerate(vectors):
        verdict, detail = judge(b, i, v)
        if verdict == "fail":
            fails.append((v["name"], detail))
        elif verdict == "escaped":
            escaped.add(v["name"])
    assert not fails, fails[:10]
    assert escaped == EXPECTED_ESCAPES


def test_vmtests_unknown_reference_output_are_excluded():
    unknown = [v["name"] for v in load_vmtests() if v["ignored"] == "reference_output_unknown"]
    assert sorted(unknown) == sorted(["jumpTo1InstructionafterJump", "sstore_load_2",
                                      "jumpi_at_the_end"])


def _run_op(op, nargs, operand_rows):
    o = OracleEVM()
    cid = o.load_code(pysem.op_program(op, nargs))
    b = LaneBatch(LaneShape(n=len(operand_rows), stack_cap=16, mem_cap=64,
                            calldata_cap=96, storage_cap=4))
    for i, row in enumerate(operand_rows):
        cd = b"".join(x.to_bytes(32, "big") for x in row)
        b.set_lane(i, code_id=cid, calldata=cd, gas_limit=10 ** 6)
    o.run(b)
    assert (b.status == MG_HALT_STOP).all()
    return [b.storage_dict(i, drop_zero=False).get(0, None) for i in range(b.n)]


@pytest.mark.parametrize("op", sorted(pysem.BINOPS))
def test_arithmetic_matches_python_restatement(op):
    nargs, fn = pysem.BINOPS[op]
    rng = random.Random(0x4D59 + op)
    sp = pysem.special_words()
    rows = [tuple(rng.choice(sp) for _ in range(nargs)) for _ in range(300)]
    rows += [tuple(rng.getrandbits(rng.choice([8, 64, 128, 255, 256])) for _ in range(nargs))
             for _ in range(300)]
    got = _run_op(op, nargs, rows)
    for row, g in zip(rows, got):
        assert g == fn(*row), (hex(op), [hex(x) for x in row], hex(g), hex(fn(*row)))


@pytest.mark.parametrize("opname,op", [("shl", 0x1B), ("shr", 0x1C), ("sar", 0x1D)])
def test_eip145_vectors(opname, op):
    vecs = load_json("shift_vectors.json")[opname]
    assert vecs
    rows = [(int(v["shift"], 16), int(v["value"], 16)) for v in vecs]
    got = _run_op(op, 2, rows)
    for v, g in zip(vecs, got):
        assert g == int(v["expected"], 16), v


def test_keccak_known_answer_and_permutation():
    kat = int(load_json("keccak_kat.json")["empty"])
    assert int.from_bytes(keccak256(b""), "big") == kat
    rng = random.Random(7)
    for n in [0, 1, 31, 32, 33, 64, 135, 136, 137, 271, 272, 1000]:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        # same permutation with the NIST pad byte must equal hashlib's SHA3-256
        assert keccak256(data, pad=0x06) == hashlib.sha3_256(data).digest()


def test_sha3_opcode_uses_keccak():
    # MSTORE(0, x) ; SHA3(0, 64) of (x, 0) ; SSTORE(0, hash)
    x = 0xDEADBEEF
    code = bytes([0x7F]) + x.to_bytes(32, "big") + bytes(
        [0x60, 0, 0x52, 0x60, 0x40, 0x60, 0, 0x20, 0x60, 0, 0x55, 0x00])
    o = OracleEVM()
    cid = o.load_code(code)
    b = LaneBatch(LaneShape(n=1, stack_cap=16, mem_cap=128, calldata_cap=32, storage_cap=4))
    b.set_lane(0, code_id=cid, gas_limit=10 ** 6)
    o.run(b)
    want = int.from_bytes(keccak256(x.to_bytes(32, "big") + bytes(32)), "big")
    assert b.storage_dict(0)[0] == want


def test_opcode_table_matches_reference():
    table = load_json("opcodes.json")
    by_byte = {d["byte"]: d for d in table.values()}
    for byte in range(256):
        info = opcode_info(byte)
        if byte not in by_byte:
            assert info is None, hex(byte)
            continue
        d = by_byte[byte]
        assert info == (d["gas"][0], d["gas"][1], d["stack"][0]), hex(byte)


def test_stack_table_quirks():
    # ADDMOD needs 2 by the table but pops 3: the pop raises instead (Appendix A #5)
    o = OracleEVM()
    cid = o.load_code(bytes([0x60, 1, 0x60, 2, 0x08, 0x00]))
    b = LaneBatch(LaneShape(n=1, stack_cap=16, mem_cap=64, calldata_cap=32, storage_cap=4))
    b.set_lane(0, code_id=cid)
    o.run(b)
    assert b.status[0] == MG_VMEXC and b.aux[0] == MG_EXC_STACK_UNDERFLOW
    assert b.pc[0] == 2 and b.gas_min[0] == 6  # pre-step state of the ADDMOD


def test_jump_resolution_first_address_at_or_above():
    # JUMP to address 3 (inside PUSH2 data) lands on the next instruction (a JUMPDEST)
    # util.py:54-58; JUMPI true to a non-JUMPDEST drops the path silently.
    code = bytes([0x60, 0x03, 0x56, 0x61, 0xAA, 0x5B, 0x60, 1, 0x60, 0, 0x55, 0x00])
    # addresses: 0 PUSH1, 2 JUMP, 3 PUSH2 (aa 5b), 6 PUSH1 ... -> 3 is the PUSH2, not JUMPDEST
    o = OracleEVM()
    cid = o.load_code(code)
    b = LaneBatch(LaneShape(n=1, stack_cap=16, mem_cap=64, calldata_cap=32, storage_cap=4))
    b.set_lane(0, code_id=cid)
    o.run(b)
    assert b.status[0] == MG_VMEXC  # invalid jump destination (PUSH2 at 3)
    # target 4 is inside PUSH2's data (addresses 4,5): the first instruction at or
    # above it is the JUMPDEST at 6, so the jump succeeds where the EVM would fail
    code2 = bytes([0x60, 0x04, 0x56, 0x61, 0xAA, 0xBB, 0x5B, 0x60, 1, 0x60, 0, 0x55, 0x00])
    cid2 = o.load_code(code2)
    b.set_lane(0, code_id=cid2)
    o.run(b)
    assert b.status[0] == MG_HALT_STOP and b.storage_dict(0) == {0: 1}


def test_disassembler_fixture_instruction_count():
    """disassembler_test.py:8-10: the reference's 3,523-instruction code (bzzr
    metadata trimmed).  Oracle and host instruction lists both have 3,523
    entries and agree instruction by instruction."""
    from mythril_amd.laser.disassembly import Disassembly
    from mythril_amd.laser.opcodes import OPCODES
    fx = load_json("disassembly.json")
    code = bytes.fromhex(fx["code"][2:])
    o = OracleEVM()
    ops, addrs = o.code_table(o.load_code(code))
    host = Disassembly(fx["code"]).instruction_list
    assert len(host) == ops.size == fx["instructions"] == 3523
    for k, ins in enumerate(host):
        assert ins["address"] == addrs[k]
        byte = OPCODES.get(ins["opcode"])
        if byte is not None:
            assert byte == ops[k], (k, ins)
