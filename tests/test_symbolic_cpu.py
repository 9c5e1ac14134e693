"""Symbolic lanes on CPU: the host half of the expression arena.

* decode_stack builds, from hand-written arena planes, exactly the expressions
  the CPU restatement (tests/symref.py) builds for the same instructions
  (hash-consed: identical constructions are the same node);
* encode_stack -> decode_stack is the identity on those expressions, shares
  repeated subterms, and refuses expressions no node produced;
* jumpi_successors forks as instructions.py:1558-1636 (both branches, the
  negated / plain condition, depth + 1, JUMPI gas, a non-JUMPDEST target keeps
  only the fall-through);
* a symbolic message call (transaction/symbolic.py:105-150) into the
  reference's flag_array and symbolic_exec_bytecode contracts through the
  batched LaserEVM ends in the same path outcomes and constraint sequences as
  the restatement (the oracle device hands every symbolic lane to the escape
  handler; tests/test_gpu_symbolic.py runs the same call on kernel 1).
"""
import pytest

import symcases
import symref
from mythril_amd import workloads
from mythril_amd.lanes import (LaneBatch, LaneShape, MG_SYM_BIN, MG_SYM_CDLOAD, MG_SYM_CDSIZE,
                               MG_SYM_CONST, MG_SYM_ENV, MG_SYM_UN, word_to_limbs)
from mythril_amd.laser import (Account, Disassembly, MessageCallTransaction, SymbolicCalldata,
                               WorldState)
from mythril_amd.laser import symbolic as sym
from mythril_amd.smt.expr import BitVec, Bool, symbol_factory
from oracle_device import OracleDevice

BVV, BVS = symbol_factory.BitVecVal, symbol_factory.BitVecSym


def _state(code_hex="00"):
    ws = WorldState()
    acct = Account(workloads.CONTRACT, code=Disassembly(code_hex))
    ws.put_account(acct)
    tx = MessageCallTransaction(world_state=ws, identifier="7", callee_account=acct,
                                caller=BVS("sender_7", 256), origin=BVS("sender_7", 256),
                                call_data=SymbolicCalldata("7"), gas_price=BVS("gas_price7", 256),
                                gas_limit=8_000_000, call_value=BVS("call_value7", 256))
    gs = tx.initial_global_state()
    gs.transaction_stack.append((tx, None))
    return gs


def _batch():
    return LaneBatch(LaneShape(n=1, stack_cap=16, node_cap=32, const_cap=16))


def test_decode_builds_the_restatements_expressions():
    s = _state()
    b = _batch()
    # node 0: CALLDATALOAD(const 4); node 1: CALLDATASIZE; node 2: CALLVALUE
    # node 3: LT(node1, const 4) (Bool); node 4: ISZERO(node3); node 5: ADD(node0, node2)
    # node 6: EQ(node5, const 4); node 7: NOT(node 0); node 8: SHR(const 224, node 0)
    b.cval[0, 0] = word_to_limbs(4)
    b.cval[0, 1] = word_to_limbs(224)
    C = MG_SYM_CONST
    rows = [(MG_SYM_CDLOAD | 256 << 8, C | 0, 0, 0), (MG_SYM_CDSIZE | 256 << 8, 0, 0, 0),
            (MG_SYM_ENV | 256 << 8, 0, 0, 3), (MG_SYM_BIN | 1 << 8, 1, C | 0, 0x10),
            (MG_SYM_UN | 256 << 8, 3, 0, 0x15), (MG_SYM_BIN | 256 << 8, 0, 2, 0x01),
            (MG_SYM_BIN | 1 << 8, 5, C | 0, 0x14), (MG_SYM_UN | 256 << 8, 0, 0, 0x19),
            (MG_SYM_BIN | 256 << 8, C | 1, 0, 0x1C)]
    for k, r in enumerate(rows):
        b.node[0, k] = r
    b.n_nodes[0], b.n_consts[0] = len(rows), 2
    b.sp[0] = len(rows) + 1
    b.stack[0, 0] = word_to_limbs(99)
    for k in range(len(rows)):
        b.stag[0, k + 1] = k + 1
    got = sym.decode_stack(b, 0, s)
    cd = s.environment.calldata
    e = symref.Engine()
    lt = e._binary(0x10, cd.size, BVV(4, 256))
    assert isinstance(lt, Bool)
    from mythril_amd.smt.expr import If
    # a Bool goes on the stack as If(b, 1, 0) (machine_state.py:39-46), and ISZERO
    # of that word is If(word == 0, 1, 0) (instructions.py:749-763)
    lt_w = If(lt, BVV(1, 256), BVV(0, 256))
    iszero = If(lt_w == 0, BVV(1, 256), BVV(0, 256))
    add = e._binary(0x01, symref._word_at(cd, BVV(4, 256)), s.environment.callvalue)
    eq_w = If(e._binary(0x14, add, BVV(4, 256)), BVV(1, 256), BVV(0, 256))
    want = [BVV(99, 256), symref._word_at(cd, BVV(4, 256)), cd.size, s.environment.callvalue, lt_w, iszero,
            add, eq_w, BVV((1 << 256) - 1, 256) - symref._word_at(cd, BVV(4, 256)),
            e._binary(0x1C, BVV(224, 256), symref._word_at(cd, BVV(4, 256)))]
    assert [x.raw for x in got] == [x.raw for x in want]
    assert [type(x) for x in got] == [type(x) for x in want]


def test_encode_decode_round_trip_and_sharing():
    s = _state()
    b = _batch()
    b.node[0, 0] = (MG_SYM_CDLOAD | 256 << 8, MG_SYM_CONST | 0, 0, 0)
    b.node[0, 1] = (MG_SYM_BIN | 256 << 8, 0, 0, 0x01)          # x + x
    b.node[0, 2] = (MG_SYM_BIN | 1 << 8, 1, MG_SYM_CONST | 1, 0x10)
    b.cval[0, 0] = word_to_limbs(0)
    b.cval[0, 1] = word_to_limbs(7)
    b.n_nodes[0], b.n_consts[0] = 3, 2
    b.sp[0] = 3
    b.stag[0, :3] = (1, 2, 3)
    stack = sym.decode_stack(b, 0, s)
    c = _batch()
    c.sp[0] = 3
    assert sym.encode_stack(c, 0, stack)
    assert int(c.n_nodes[0]) == 3            # x shared by both operands of x + x
    again = sym.decode_stack(c, 0, s)
    assert [x.raw for x in again] == [x.raw for x in stack]
    # a term no node produced rides on the lane as an opaque node (MG_SYM_TERM)
    fresh = [BVS("fresh_from_elsewhere", 256), stack[1] + BVS("fresh_from_elsewhere", 256)]
    d = _batch()
    d.sp[0] = 2
    assert sym.encode_stack(d, 0, fresh)
    assert [x.raw for x in sym.decode_stack(d, 0, s)] == [x.raw for x in fresh]
    assert sym.lane_eligible(_with_stack(s, fresh))
    assert sym.lane_eligible(_with_stack(s, stack))


def _with_stack(s, stack):
    from copy import copy
    from mythril_amd.laser.state import MachineStack
    t = copy(s)
    t.mstate.stack = MachineStack(list(stack))
    return t


def test_jumpi_successors_follow_the_reference():
    # PUSH1 5, JUMPI, STOP, STOP, JUMPDEST (byte 5), STOP
    s = _state("60055700005b00")
    cond = s.environment.calldata.size
    s.mstate.stack.append(cond)
    s.mstate.stack.append(BVV(5, 256))
    s.mstate.pc = 1
    out = sym.jumpi_successors(s)
    assert len(out) == 2
    fall, jump = out
    assert fall.mstate.pc == 2 and fall.world_state.constraints[-1].raw is (cond == 0).raw
    assert jump.get_current_instruction()["opcode"] == "JUMPDEST"
    assert jump.world_state.constraints[-1].raw is (cond != 0).raw
    for t in out:
        assert t.mstate.depth == s.mstate.depth + 1 and len(t.mstate.stack) == 0
        assert t.mstate.min_gas_used == s.mstate.min_gas_used + 10
    s.mstate.stack[-1] = BVV(3, 256)                            # not a JUMPDEST: no jump branch
    assert len(sym.jumpi_successors(s)) == 1
    from mythril_amd.smt.expr import Not
    s.mstate.stack[-2] = cond < BVV(3, 256)                     # a Bool condition: Not(c) / c
    s.mstate.stack[-1] = BVV(5, 256)
    fall, jump = sym.jumpi_successors(s)
    assert fall.world_state.constraints[-1].raw is Not(cond < BVV(3, 256)).raw
    assert jump.world_state.constraints[-1].raw is (cond < BVV(3, 256)).raw


@pytest.mark.parametrize("name", symcases.ALL_CASES)
def test_symbolic_call_outcomes_equal_the_restatement(name, monkeypatch):
    got, want, laser = symcases.run_both(OracleDevice(), name, monkeypatch)
    assert sum(want.values()) >= (2 if name in symcases.FIELD else 5 if name in symcases.SYNTH else 7)
    assert got == want


@pytest.mark.parametrize("name", symcases.SYM_CREATIONS_ALL)
def test_symbolic_creation_outcomes_equal_the_restatement(name, monkeypatch):
    """transaction/symbolic.py's creation (symbolic calldata: CODESIZE + 0x200
    pins its size, constructor arguments come from CODECOPY past the end of
    the code) through LaserEVM: the oracle device escapes every symbolic lane
    to the restatement, so this pins the harness the GPU test uses."""
    got, want, laser = symcases.run_creation_both(OracleDevice(), name, monkeypatch)
    assert sum(want.values()) >= 2
    assert got == want


def test_restated_creation_calldata_opcodes_follow_the_reference():
    """instructions.py:878-891 / 979-1000 / 1074-1104 on a creation with
    symbolic calldata: CALLDATACOPY pops three words and copies nothing;
    CODESIZE = code size + 0x200 with calldata.size == it appended; CODECOPY
    from past the end of the code copies calldata[offset - code size + k]."""
    from mythril_amd.laser import ContractCreationTransaction, Disassembly, SymbolicCalldata, WorldState
    # PUSH1 8 PUSH1 0 PUSH1 0 CALLDATACOPY | CODESIZE | PUSH1 3 PUSH1 0x13 PUSH1 0x40 CODECOPY | STOP
    code = bytes.fromhex("600860006000" "37" "38" "6003601360403900")
    ws = WorldState()
    tx = ContractCreationTransaction(world_state=ws, identifier="77", gas_price=0, gas_limit=8_000_000,
                                     origin=1, code=Disassembly(code), caller=1,
                                     call_data=SymbolicCalldata("77"), call_value=0)
    s = tx.initial_global_state()
    s.transaction_stack.append((tx, None))
    e = symref.Engine()
    for _ in range(4):
        (s,) = e.step(s)
    assert len(s.mstate.stack) == 0 and len(s.mstate.memory) == 0          # CALLDATACOPY: nothing
    (s,) = e.step(s)
    n = len(code) + 0x200
    assert s.mstate.stack[-1].value == n
    cd = s.environment.calldata
    assert s.world_state.constraints[-1].raw is (cd.size == BVV(n, 256)).raw
    for _ in range(4):
        (s,) = e.step(s)
    mem = s.mstate.memory
    assert len(mem) == 0x60
    assert {p: x.raw for p, x in mem.symbolic_bytes().items()} == \
        {0x40 + k: cd[0x13 - len(code) + k].raw for k in range(3)} if 0x13 >= len(code) else True


def test_restated_symbolic_exp_follows_the_reference():
    """exp_ (instructions.py:624-638) of a symbolic exponent: Power(256, x) on the
    stack and exponent_function_manager's condition (Power > 0, the 256**i table,
    periodicity mod 32 for base 256) appended; the device's EXP node decodes to
    the same term and re-encodes as SYM_BIN 0x0a."""
    from mythril_amd.smt.exponent_manager import exponent_function_manager
    s = _state("600035" "610100" "0a" "00")          # PUSH1 0 CALLDATALOAD PUSH2 0x100 EXP STOP
    e = symref.Engine()
    for _ in range(4):
        (s,) = e.step(s)
    x = s.environment.calldata.get_word_at(0)
    want, cond = exponent_function_manager.create_condition(BVV(256, 256), x)
    assert s.mstate.stack[-1].raw is want.raw
    assert s.world_state.constraints[-1].raw is cond.raw
    got = sym.binary(0x0A, BVV(256, 256), x)
    assert got.raw is want.raw


# ---- symbolic memory, storage chains and SHA3 (ABI v7) -----------------------------
def _run_restatement(code_hex, steps):
    s = _state(code_hex)
    s.environment.active_account.storage.to_chain()
    e = symref.Engine()
    for _ in range(steps):
        (s,) = e.step(s)
    return s


# PUSH1 4 CALLDATALOAD | PUSH1 0 MSTORE | PUSH1 0x20 PUSH1 0 SHA3 | DUP1 PUSH1 1 SSTORE |
# SLOAD | PUSH1 0x10 MLOAD | STOP
_MEMPROG = "600435" "600052" "6020600020" "80600155" "54" "601051" "00"


def test_restated_memory_storage_and_sha3_follow_the_reference():
    s = _run_restatement(_MEMPROG, 13)
    cd = s.environment.calldata
    x = cd.get_word_at(BVV(4, 256))
    from mythril_amd.smt.expr import Concat, Extract, Function, K, Node, _select
    k = Function("keccak256_256", [256], 256)(x)                 # 32 bytes of one word: x itself
    chain = Node("store", 0, (K(256, 256, 0).raw, BVV(1, 256).raw, k.raw), (256, 256))
    sel = _select(chain, k.raw)
    assert sel.op == "select" and sel.args[0] is chain           # 1 vs k: z3 cannot decide
    word = Concat(Extract(127, 0, x), BVV(0, 128))               # bytes 16..47: half of x, then zeros
    assert [w.raw for w in s.mstate.stack] == [sel, word.raw]
    assert s.mstate.memory.get_word_at(0).raw is x.raw
    st = s.environment.active_account.storage
    assert [(a.raw, b.raw) for a, b in st.chain()] == [(BVV(1, 256).raw, k.raw)]
    assert st[BVV(1, 256)].raw is k.raw and st[k].raw is sel and st[BVV(2, 256)].value == 0


def test_lane_encoding_of_memory_and_storage_round_trips():
    s = _run_restatement(_MEMPROG, 13)
    le = sym.encode_state(s)
    assert le.symbolic and le.store is not None and len(le.mem) == 32
    b = LaneBatch(LaneShape(n=1, stack_cap=16, node_cap=128, const_cap=32))
    le.write(b, 0)
    b.sp[0] = len(s.mstate.stack)
    b.msize[0] = len(s.mstate.memory)
    b.flags[0] = le.flags
    stack, mem, storage = sym.decode_lane(b, 0, s)
    assert [w.raw for w in stack] == [w.raw for w in s.mstate.stack]
    assert {p: e.raw for p, e in mem.symbolic_bytes().items()} == \
        {p: e.raw for p, e in s.mstate.memory.symbolic_bytes().items()}
    assert [(a.raw, c.raw) for a, c in storage.chain()] == \
        [(a.raw, c.raw) for a, c in s.environment.active_account.storage.chain()]
    assert storage.chain_raw() is s.environment.active_account.storage.chain_raw()
    # decoding with the encoder's terms as the arena prefix (what _materialise does
    # for a lane it packed) gives every node the same term and type as rebuilding it
    full, pre = sym._Decoder(b, 0, s), sym._Decoder(b, 0, s, le.enc.node_raw)
    for k in range(int(b.n_nodes[0])):
        x, y = full.node(k), pre.node(k)
        assert x.raw is y.raw and type(x) is type(y), k
    st2, mem2, sto2 = sym.decode_lane(b, 0, s, le.enc.node_raw)
    assert [(type(w), w.raw) for w in st2] == [(type(w), w.raw) for w in stack]
    assert [(a.raw, c.raw) for a, c in sto2.chain()] == [(a.raw, c.raw) for a, c in storage.chain()]


def test_device_memory_parts_decode_to_the_reference_word():
    """The parts kernel 1 builds for a memory read (EXTRACT / CONCAT nodes, a
    constant run) decode to simplify(Concat(bytes)) of the same bytes."""
    s = _state()
    b = _batch()
    C = MG_SYM_CONST
    from mythril_amd.lanes import MG_SYM_CONCAT, MG_SYM_EXTRACT, MG_SYM_KECCAK
    b.cval[0, 0] = word_to_limbs(4)
    b.cval[0, 1] = word_to_limbs(0xABCD)
    b.node[0, 0] = (MG_SYM_CDLOAD | 256 << 8, C | 0, 0, 0)
    b.node[0, 1] = (MG_SYM_EXTRACT | 128 << 8, 0, 0, (127 << 16) | 0)        # bytes 16..31 of x
    b.node[0, 2] = (MG_SYM_CONCAT | 256 << 8, 1, C | 1, 128 | (128 << 16))   # then 16 bytes 0..0abcd
    b.node[0, 3] = (MG_SYM_KECCAK | 256 << 8, 2, 0, 256)
    b.n_nodes[0], b.n_consts[0] = 4, 2
    b.sp[0] = 2
    b.stag[0, 0], b.stag[0, 1] = 3, 4
    word, h = sym.decode_stack(b, 0, s)
    mem = s.mstate.memory
    mem.extend(64)
    x = s.environment.calldata.get_word_at(BVV(4, 256))
    mem.write_word_at(0, x)
    mem.write_word_at(32, BVV(0xABCD << 128, 256))           # bytes 32..47 end in ab cd
    assert word.raw is mem.get_word_at(16).raw
    from mythril_amd.smt.keccak_manager import KeccakFunctionManager
    assert h.raw is KeccakFunctionManager().create_keccak(mem.get_word_at(16)).raw


def test_restated_symbolic_calldata_copy_follows_the_reference():
    """_calldata_copy_helper (instructions.py:807-860) with a symbolic size and a
    symbolic calldata offset: 320 bytes (SYMBOLIC_CALLDATA_SIZE), byte k =
    calldata[simplify(offset + k)]; the arena's MG_SYM_CDBYTEX nodes decode to
    the same bytes.  A symbolic memory offset copies nothing."""
    from mythril_amd.lanes import MG_SYM_CDBYTEX, MG_SYM_CDLOAD
    # CALLDATASIZE | PUSH1 4 CALLDATALOAD | PUSH1 0x80 CALLDATACOPY | STOP
    s = _run_restatement("36" "600435" "608037" "00", 5)
    cd = s.environment.calldata
    x = cd.get_word_at(BVV(4, 256))
    mem = s.mstate.memory
    assert len(mem) == (0x80 + 320 + 31) // 32 * 32 and len(s.mstate.stack) == 0
    got = mem.symbolic_bytes()
    assert sorted(got) == list(range(0x80, 0x80 + 320))
    for k in (0, 1, 2, 31, 319):
        assert got[0x80 + k].raw is cd[sym.cd_index(x, k)].raw
    assert sym.cd_index(x, 2).raw is sym.cd_index(sym.cd_index(x, 1), 1).raw
    # the device's form: CDLOAD(4) then 320 CDBYTEX nodes on it
    b = _batch()
    b.node[0, 0] = (MG_SYM_CDLOAD | 256 << 8, MG_SYM_CONST | 0, 0, 0)
    b.cval[0, 0] = word_to_limbs(4)
    for k in range(3):
        b.node[0, 1 + k] = (MG_SYM_CDBYTEX | 8 << 8, 0, 0, k)
    b.n_nodes[0], b.n_consts[0] = 4, 1
    dec = sym._Decoder(b, 0, s)
    for k in range(3):
        assert dec.node(1 + k).raw is got[0x80 + k].raw
    # re-encoding a byte replays its provenance: node (CDBYTEX, offset node, k)
    enc = sym._Encoder()
    t = enc.byte(dec.node(3))
    assert enc.nodes[(t - 1) >> 5][0] & 0xFF == MG_SYM_CDBYTEX and enc.nodes[(t - 1) >> 5][3] == 2
    # a symbolic memory offset: the copy is dropped, the operands popped
    s2 = _run_restatement("6020" "6000" "600035" "37" "00", 5)     # PUSH1 32 PUSH1 0 (PUSH1 0 CALLDATALOAD) CALLDATACOPY
    assert len(s2.mstate.stack) == 0 and len(s2.mstate.memory) == 0


def test_memory_at_symbolic_keys_round_trips_and_decodes_like_the_byte_map():
    """MSTORE / MSTORE8 / MLOAD at symbolic offsets (memory.py:117-203): the
    restatement's byte map keyed by simplify(index) survives encode -> lane ->
    decode as MG_SYM_MSTOREK events, and the device's event + MLOADK nodes decode
    to what the byte map gives."""
    from mythril_amd.lanes import MG_SYM_BIN, MG_SYM_CDLOAD, MG_SYM_MLOADK, MG_SYM_MSTOREK
    from mythril_amd.laser.state import Memory
    from mythril_amd.smt.expr import Extract
    # PUSH1 4 CALLDATALOAD (x) | PUSH2 0x1234 DUP2 MSTORE | PUSH1 0x20 CALLDATALOAD DUP2 PUSH1 0x28 ADD
    # MSTORE8 | DUP1 PUSH1 0x10 ADD MLOAD | STOP
    code = "600435" "611234" "81" "52" "602035" "81" "6028" "01" "53" "80" "6010" "01" "51" "00"
    s = _run_restatement(code, 14)
    mem = s.mstate.memory
    assert mem.symbolic_keys and len(mem.symbolic_key_bytes()) == 33
    le = sym.encode_state(s)
    b = LaneBatch(LaneShape(n=1, stack_cap=16, node_cap=256, const_cap=64, mem_cap=64))
    le.write(b, 0)
    b.sp[0] = len(s.mstate.stack)
    b.msize[0] = len(mem)
    b.flags[0] = le.flags
    stack, mem2, _ = sym.decode_lane(b, 0, s)
    assert [w.raw for w in stack] == [w.raw for w in s.mstate.stack]
    want = {k: (v if isinstance(v, int) else v.raw) for k, v in mem.symbolic_key_bytes().items()}
    got = {k: (v if isinstance(v, int) else v.raw) for k, v in mem2.symbolic_key_bytes().items()}
    assert got == want and list(got) == list(want)
    # the device's form: x = CDLOAD(4); write 0x1234 at x; read at x; read at x + 16
    c = LaneBatch(LaneShape(n=1, stack_cap=16, node_cap=16, const_cap=8))
    c.node[0, 0] = (MG_SYM_CDLOAD | 256 << 8, MG_SYM_CONST | 0, 0, 0)
    c.node[0, 1] = (MG_SYM_MSTOREK, 0, MG_SYM_CONST | 1, 1)
    c.node[0, 2] = (MG_SYM_MLOADK | 256 << 8, 0, 0, 0)
    c.node[0, 3] = (MG_SYM_BIN | 256 << 8, 0, MG_SYM_CONST | 2, 0x01)
    c.node[0, 4] = (MG_SYM_MLOADK | 256 << 8, 3, 0, 0)
    c.node[0, 5] = (MG_SYM_MSTOREK, 3, 0, 2)                   # MSTORE8 of x's low byte at x + 16
    c.node[0, 6] = (MG_SYM_MLOADK | 256 << 8, 0, 0, 0)
    for k, v in enumerate((4, 0x1234, 16)):
        c.cval[0, k] = word_to_limbs(v)
    c.n_nodes[0], c.n_consts[0] = 7, 3
    dec = sym._Decoder(c, 0, s)
    x = s.environment.calldata.get_word_at(BVV(4, 256))
    ref = Memory()
    ref.write_word_at(x, BVV(0x1234, 256))
    assert dec.node(2).raw is ref.get_word_at(x).raw and dec.node(2).value == 0x1234
    assert dec.node(4).raw is ref.get_word_at(x + BVV(16, 256)).raw
    ref[x + BVV(16, 256)] = Extract(7, 0, x)
    assert dec.node(6).raw is ref.get_word_at(x).raw and dec.node(6).symbolic
    full = sym._Decoder(c, 0, s).memory()
    assert {k: (v if isinstance(v, int) else v.raw) for k, v in full.symbolic_key_bytes().items()} == \
        {k: (v if isinstance(v, int) else v.raw) for k, v in ref.symbolic_key_bytes().items()}


def test_sha3_at_a_symbolic_offset_decodes_to_the_hash_of_the_byte_map():
    """sha3_ (instructions.py:1014-1051) at a symbolic offset and concrete length:
    the device's MLOADK range node (w = length) under a KECCAK node decodes to
    keccak over simplify(Concat(memory[offset:offset + length])) of the byte map
    the MSTOREK events before it built; the restatement hashes the same data."""
    from mythril_amd.lanes import MG_SYM_CDLOAD, MG_SYM_KECCAK, MG_SYM_MLOADK, MG_SYM_MSTOREK
    from mythril_amd.laser.state import Memory
    c = LaneBatch(LaneShape(n=1, stack_cap=16, node_cap=16, const_cap=8))
    c.node[0, 0] = (MG_SYM_CDLOAD | 256 << 8, MG_SYM_CONST | 0, 0, 0)
    c.node[0, 1] = (MG_SYM_MSTOREK, 0, MG_SYM_CONST | 1, 1)              # MSTORE(x, 0x1234)
    c.node[0, 2] = (MG_SYM_MLOADK | (8 * 40) << 8, 0, 0, 40)             # memory[x:x+40]
    c.node[0, 3] = (MG_SYM_KECCAK | 256 << 8, 2, 0, 8 * 40)
    c.node[0, 4] = (MG_SYM_MSTOREK, 0, 0, 1)                             # MSTORE(x, x)
    c.node[0, 5] = (MG_SYM_MLOADK | (8 * 32) << 8, 0, 0, 32)
    c.node[0, 6] = (MG_SYM_KECCAK | 256 << 8, 5, 0, 8 * 32)
    for k, v in enumerate((4, 0x1234)):
        c.cval[0, k] = word_to_limbs(v)
    c.n_nodes[0], c.n_consts[0] = 7, 2
    s = _run_restatement("5b00", 1)
    dec = sym._Decoder(c, 0, s)
    x = s.environment.calldata.get_word_at(BVV(4, 256))
    ref = Memory()
    ref.write_word_at(x, BVV(0x1234, 256))

    def data(n):
        return data_at(ref, x, n)
    assert dec.node(2).raw is data(40).raw and dec.node(2).size() == 320
    assert dec.node(3).raw is sym.keccak_of(data(40)).raw and not dec.node(3).symbolic
    ref.write_word_at(x, x)
    assert dec.node(5).raw is data(32).raw and dec.node(6).raw is sym.keccak_of(data(32)).raw
    assert dec.node(6).symbolic
    # the restatement at the same point: x = CALLDATALOAD(4); MSTORE(x, 0x1234); SHA3(x, 40)
    s2 = _run_restatement("600435" "611234" "81" "52" "6028" "81" "20" "00", 8)
    top = s2.mstate.stack[-1]
    assert top.raw is sym.keccak_of(data_at(s2.mstate.memory, x, 40)).raw


def data_at(mem, x, n):
    """simplify(Concat(memory[x:x+n])) as sha3_ builds it (instructions.py:1036-1045)."""
    from mythril_amd.smt.expr import simplify_concat
    return simplify_concat([b if isinstance(b, BitVec) else BVV(b, 8) for b in mem[x: x + BVV(n, 256)]])


def test_selfbalance_node_and_symbolic_return_range():
    """selfbalance_ (instructions.py:968-976): a lane whose active account's
    balance is symbolic carries MG_LANE_SYMBAL, and the device's MG_SYM_ENV node
    with w = MG_ENV_SELFBALANCE decodes to environment.active_account.balance()
    with no provenance (a later re-encode keeps the term itself).  A RETURN /
    REVERT of a symbolic range halts with ret_len = MG_RET_SYMBOLIC: no return
    data bytes (tests/symref.py ends such a transaction with return_data=None)."""
    from mythril_amd.lanes import MG_ENV_SELFBALANCE, MG_LANE_SYMBAL, MG_RET_SYMBOLIC, MG_SYM_ENV
    s = _run_restatement("47" "00", 1)                                 # SELFBALANCE STOP
    bal = s.environment.active_account.balance()
    assert bal.symbolic and s.mstate.stack[-1].raw is bal.raw
    le = sym.encode_state(s)
    assert le.flags & MG_LANE_SYMBAL
    c = _batch()
    c.node[0, 0] = (MG_SYM_ENV | 256 << 8, 0, 0, MG_ENV_SELFBALANCE)
    c.n_nodes[0] = 1
    assert sym._Decoder(c, 0, s).node(0).raw is bal.raw
    assert sym._PROV.get(bal.raw) is None or sym._PROV[bal.raw][0] != MG_SYM_ENV
    c.ret_offset[0], c.ret_len[0] = 0, MG_RET_SYMBOLIC
    assert c.return_data(0) is None
    c.ret_len[0] = 2
    assert c.return_data(0) == b"\x00\x00"


def test_returndatasize_node_decodes_to_the_last_return_data_size():
    """returndatasize_ (instructions.py:1359-1370) after a host CALL that left a
    symbolic size: the lane carries MG_LANE_SYMRDS and the device's MG_SYM_ENV node
    (w = MG_ENV_RETURNDATASIZE) decodes to last_return_data.size."""
    from mythril_amd.lanes import MG_ENV_RETURNDATASIZE, MG_LANE_SYMRDS, MG_SYM_ENV
    s = _run_restatement("6000" "35" "00", 2)                           # a symbolic lane
    rds = s.new_bitvec("returndatasize", 256)
    s.last_return_data = symref.ReturnData([], rds)
    assert sym.encode_state(s).flags & MG_LANE_SYMRDS
    c = _batch()
    c.node[0, 0] = (MG_SYM_ENV | 256 << 8, 0, 0, MG_ENV_RETURNDATASIZE)
    c.n_nodes[0] = 1
    assert sym._Decoder(c, 0, s).node(0).raw is rds.raw
    s.last_return_data = None
    assert not sym.encode_state(s).flags & MG_LANE_SYMRDS


def test_balance_node_decodes_like_balance_():
    """balance_ (instructions.py:907-931) with no dynamic loader: the device's
    MG_SYM_BALANCE node over a known concrete address decodes to that account's
    balance(), over a symbolic or unknown address to the If chain over the world
    state's accounts -- the restatement's value for the same instruction."""
    from mythril_amd.lanes import MG_SYM_BALANCE
    s = _run_restatement("30" "31" "6000" "35" "31" "611234" "31" "00", 7)
    want = [x.raw for x in s.mstate.stack]
    c = _batch()
    c.node[0, 0] = (MG_SYM_CDLOAD | 256 << 8, MG_SYM_CONST | 1, 0, 0)
    c.node[0, 1] = (MG_SYM_BALANCE | 256 << 8, MG_SYM_CONST | 0, 0, 0)
    c.node[0, 2] = (MG_SYM_BALANCE | 256 << 8, 0, 0, 0)
    c.node[0, 3] = (MG_SYM_BALANCE | 256 << 8, MG_SYM_CONST | 2, 0, 0)
    for k, v in enumerate((workloads.CONTRACT, 0, 0x1234)):
        c.cval[0, k] = word_to_limbs(v)
    c.n_nodes[0], c.n_consts[0] = 4, 3
    dec = sym._Decoder(c, 0, s)
    assert [dec.node(k).raw for k in (1, 2, 3)] == want


def test_symlen_record_parses_and_restates_sha3_of_a_symbolic_length():
    """MG_REC_SYMLEN (sha3_ of a symbolic length, instructions.py:1023-1028): the
    record parses to (step, "symlen", node, 64), and the restatement takes the
    length as 64 with `n == 64` appended before the hash of memory[index:+64]."""
    from mythril_amd.lanes import MG_REC_HEADER, MG_REC_SYMLEN
    b = LaneBatch(LaneShape(n=1, stack_cap=16, rec_cap=64))
    b.rec[0, :MG_REC_HEADER + 1] = [MG_REC_SYMLEN, 64, 3] + [0] * 8 + [5]
    b.rec_len[0] = MG_REC_HEADER + 1
    assert b.records(0) == [(3, "symlen", 5, 64)]
    # x = CALLDATALOAD(0); MSTORE(0, x); SHA3(0, CALLDATALOAD(32)); STOP
    s = _run_restatement("6000" "35" "80" "6000" "52" "6020" "35" "6000" "20" "00", 9)
    n = s.environment.calldata.get_word_at(BVV(32, 256))
    assert s.world_state.constraints[-1].raw is (n == 64).raw
    assert s.mstate.stack[-1].symbolic and len(s.mstate.memory) == 64


def test_fresh_variable_and_block_nodes_decode_like_the_restatement():
    """gas_ / coinbase_ / timestamp_ / difficulty_ (instructions.py:1386-1425,
    1700-1709) push the transaction's fresh variable of that name; number_ /
    chainid_ (:958-965, 1406-1413) the environment's words.  The device's
    MG_SYM_ENV nodes (MG_ENV_GAS .. MG_ENV_CHAINID) decode to the same terms the
    restatement pushes, and a default Environment marks the lane MG_LANE_SYMBLOCK."""
    from mythril_amd.lanes import (MG_ENV_CHAINID, MG_ENV_COINBASE, MG_ENV_DIFFICULTY, MG_ENV_GAS,
                                   MG_ENV_NUMBER, MG_ENV_TIMESTAMP, MG_LANE_SYMBLOCK, MG_SYM_ENV)
    # GAS COINBASE TIMESTAMP DIFFICULTY NUMBER CHAINID (PUSH1 0 CALLDATALOAD: a symbolic lane) STOP
    s = _run_restatement("5a" "41" "42" "44" "43" "46" "6000" "35" "00", 8)
    want = [x.raw for x in s.mstate.stack[:6]]
    assert sym.encode_state(s).flags & MG_LANE_SYMBLOCK
    c = _batch()
    for k, w in enumerate((MG_ENV_GAS, MG_ENV_COINBASE, MG_ENV_TIMESTAMP, MG_ENV_DIFFICULTY, MG_ENV_NUMBER,
                           MG_ENV_CHAINID)):
        c.node[0, k] = (MG_SYM_ENV | 256 << 8, 0, 0, w)
    c.n_nodes[0] = 6
    dec = sym._Decoder(c, 0, s)
    assert [dec.node(k).raw for k in range(6)] == want
