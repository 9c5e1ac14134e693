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
from mythril_amd.smt.expr import Bool, symbol_factory
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
    with pytest.raises(sym.NotEncodable):
        sym.encode_stack(c, 0, [BVS("fresh_from_elsewhere", 256)])
    assert not sym.lane_eligible(_with_stack(s, [BVS("fresh_from_elsewhere", 256)]))
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


@pytest.mark.parametrize("name", sorted(symcases.CONTRACTS))
def test_symbolic_call_outcomes_equal_the_restatement(name, monkeypatch):
    got, want, laser = symcases.run_both(OracleDevice(), name, monkeypatch)
    assert sum(want.values()) >= 7
    assert got == want
