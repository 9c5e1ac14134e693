"""Symbolic lanes on an MI355X: k_sym_step + the expression arena.

* co-simulation: every path of a symbolic message call into the reference's
  flag_array and symbolic_exec_bytecode contracts is stepped on the device
  until it stops (MG_FORK at a symbolic JUMPI, MG_ESCAPE, a halt); the CPU
  restatement (tests/symref.py) steps the same state the same number of
  instructions, and the decoded device stack must be the restatement's stack
  node for node (hash-consed expressions), with pc, gas, depth, memory and
  storage equal; at MG_FORK both sides fork into the same successors;
* end to end: the batched LaserEVM on kernel 1 ends the calls in the same path
  outcomes and constraint sequences as the restatement, with the symbolic
  lanes' instructions executed on the device.
"""
from copy import copy

import pytest

import symcases
import symref
from mythril_amd.device import GpuDevice
from mythril_amd.lanes import (MG_ESC_SYMBOLIC, MG_ESCAPE, MG_FORK, MG_LANE_SYMBOLIC, MG_RUNNING,
                               LaneBatch)
from mythril_amd.laser import (BreadthFirstSearchStrategy, LaserEVM, MessageCallTransaction,
                               SymbolicCalldata)
from mythril_amd.laser import symbolic as sym
from mythril_amd.laser.transaction import ACTORS
from mythril_amd.smt.exponent_manager import exponent_function_manager
from mythril_amd.smt.expr import Or, symbol_factory

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


def _initial(ws, addr, txid="50"):
    sender = symbol_factory.BitVecSym(f"sender_{txid}", 256)
    tx = MessageCallTransaction(world_state=ws, identifier=txid,
                                gas_price=symbol_factory.BitVecSym(f"gas_price{txid}", 256),
                                gas_limit=8_000_000, origin=sender, caller=sender,
                                callee_account=ws[addr], call_data=SymbolicCalldata(txid),
                                call_value=symbol_factory.BitVecSym(f"call_value{txid}", 256))
    gs = tx.initial_global_state()
    gs.transaction_stack.append((tx, None))
    gs.world_state.constraints.append(
        Or(*[tx.caller == symbol_factory.BitVecVal(a, 256) for a in ACTORS.values()]))
    return gs


def _min_forks(name: str) -> int:
    # memjump: two branches past its escaped jump; balance_of: its third JUMPI
    # tests BALANCE(0x1234) of an account the world state lacks, which the
    # host's decode folds to 0 -- a concrete JUMPI there, not a fork (svm.py
    # routes a device fork whose condition folds to a constant as an escape)
    return 1 if name in symcases.FIELD else 2 if name in ("memjump", "balance_of") else 3


@pytest.mark.parametrize("name", symcases.ALL_CASES)
def test_device_symbolic_lanes_cosimulate_with_the_restatement(dev, name):
    ws, addr = symcases.deploy(dev, name)
    vm = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy)
    queue = [_initial(ws, addr)]
    eng = symref.Engine()
    forks = device_steps = checked = sym_sha3 = halts_past_sha3 = sym_exp = 0
    while queue:
        batch_states = queue[:256]
        queue = queue[256:]
        shape = vm._shape(batch_states)
        b = LaneBatch(shape)
        for i, s in enumerate(batch_states):
            vm._pack(b, i, s)
            b.steps[i] = 0
        dev.alloc(shape)
        dev.upload(b)
        dev.step()
        dev.download(b)
        for i, s0 in enumerate(batch_states):
            n = int(b.steps[i])
            device_steps += n
            st = int(b.status[i])
            got = vm._materialise(b, i, copy(s0))
            # the path constraints LaserEVM's record replay appends (EXP: the
            # exponent manager's condition, instructions.py:624-638), in order
            for r in b.records(i):
                if r[1] == "symexp":
                    _, cond = exponent_function_manager.create_condition(*sym.exp_operands(b, i, got, r[2]))
                    got.world_state.constraints.append(cond)
                elif r[1] == "exp":
                    _, cond = exponent_function_manager.create_condition(
                        symbol_factory.BitVecVal(r[2], 256), symbol_factory.BitVecVal(r[3], 256))
                    got.world_state.constraints.append(cond)
                elif r[1] == "symlen":          # sha3_ of a symbolic length (:1023-1028)
                    got.world_state.constraints.append(sym.decode_node(b, i, got, r[2]) == r[3])
            # the restatement: the same state, the same number of instructions (a
            # halt or VmException counts as a step but leaves the state at its start)
            ref = s0
            for _ in range(n - (1 if st in (1, 2, 3, 5, 6) else 0)):
                out = eng.step(ref)
                assert len(out) == 1, (name, "the restatement forked or ended inside a device run")
                ref = out[0]
            assert got.mstate.pc == ref.mstate.pc
            assert [x.raw for x in got.mstate.stack] == [x.raw for x in ref.mstate.stack], (name, got.mstate.pc)
            assert [type(x) for x in got.mstate.stack] == [type(x) for x in ref.mstate.stack]
            assert (got.mstate.min_gas_used, got.mstate.max_gas_used, got.mstate.depth) == \
                (ref.mstate.min_gas_used, ref.mstate.max_gas_used, ref.mstate.depth)
            assert got.mstate.memory.raw() == ref.mstate.memory.raw()
            assert {p: e.raw for p, e in got.mstate.memory.symbolic_bytes().items()} == \
                {p: e.raw for p, e in ref.mstate.memory.symbolic_bytes().items()}
            # bytes at symbolic keys (MG_SYM_MSTOREK events), values and write order
            assert [(k, v if isinstance(v, int) else v.raw)
                    for k, v in got.mstate.memory.symbolic_key_bytes().items()] == \
                [(k, v if isinstance(v, int) else v.raw) for k, v in ref.mstate.memory.symbolic_key_bytes().items()]
            gst, rst = got.environment.active_account.storage, ref.environment.active_account.storage
            if rst.is_chain:
                assert [(k.raw, v.raw) for k, v in gst.chain()] == [(k.raw, v.raw) for k, v in rst.chain()]
            else:
                assert gst.slots() == rst.slots()
            recs = b.records(i)
            sym_sha3 += sum(1 for r in recs if r[1] == "symkeccak")
            sym_exp += sum(1 for r in recs if r[1] == "symexp")
            if st in (1, 2, 3) and any(r[1] == "symkeccak" for r in recs):
                halts_past_sha3 += 1
            checked += 1
            if st == MG_FORK:
                forks += 1
                mine = sym.jumpi_successors(got)
                theirs = eng.step(ref)
                assert [(t.mstate.pc, tuple(c.raw for c in t.world_state.constraints)) for t in mine] == \
                    [(t.mstate.pc, tuple(c.raw for c in t.world_state.constraints)) for t in theirs]
                queue.extend(t for t in mine if sym.lane_eligible(t))
            elif st == MG_ESCAPE:
                assert (int(b.aux[i]) >> 8) in (MG_ESC_SYMBOLIC, 1, 2, 3, 4, 8)
                if name == "memjump":
                    # the host takes the jump (as LaserEVM's escape handler would):
                    # the paths past it come back to the device
                    queue.extend(t for t in eng.step(got) if sym.lane_eligible(t))
    assert forks >= _min_forks(name) and device_steps > (10 if name in symcases.SYNTH or name in symcases.FIELD else 100) and checked > forks
    if name == "flag_array.sol.o":
        # _flags[idx]: EXP(256, idx % 32) of a symbolic index runs on the device
        assert sym_exp > 0
    if name == "overflow.sol.o":
        # symbolic storage and mapping slots: paths hash a symbolic caller (a
        # SHA3 of symbolic memory), read and write the symbolic storage and halt
        # on the device
        assert sym_sha3 > 0 and halts_past_sha3 > 0, (sym_sha3, halts_past_sha3)
    if name == "symlen_sha3":
        # SHA3 of a symbolic length: the record that pins it to 64 precedes its keccak
        assert sym_sha3 > 0, sym_sha3
    if name == "symkey_sha3":
        # SHA3 over memory at a symbolic offset: an MLOADK range node under KECCAK
        assert sym_sha3 > 0 and halts_past_sha3 > 0, (sym_sha3, halts_past_sha3)


# what a symbolic lane still hands to the host: the call family and SELFDESTRUCT
# (the reference's world-state transitions).  RETURN / REVERT of a symbolic range,
# SELFBALANCE, BALANCE (no dynamic loader), RETURNDATASIZE of a host CALL's
# symbolic size, RETURNDATACOPY of a symbolic operand and symbolic jump targets run
# on the device (ABI v14).
HOST_OPS = {"CALL", "CALLCODE", "DELEGATECALL", "STATICCALL", "CREATE", "CREATE2", "SELFDESTRUCT"}
# and, in the other reference codes, reads of other accounts' code and of environment
# words that are not fresh variables (extcodesize_ .. basefee_, instructions.py:935-1071,
# 1372-1413); GAS, COINBASE, TIMESTAMP and DIFFICULTY push fresh variables on the device
WORLD_READS = {"EXTCODESIZE", "EXTCODECOPY", "EXTCODEHASH", "BLOCKHASH", "NUMBER", "CHAINID", "BASEFEE"}


@pytest.mark.parametrize("name", symcases.ALL_CASES)
def test_symbolic_call_on_kernel1_equals_the_restatement(dev, name, monkeypatch):
    got, want, laser = symcases.run_both(dev, name, monkeypatch)
    assert got == want
    assert laser.forks >= _min_forks(name) and \
        laser.lane_steps > (10 if name in symcases.SYNTH or name in symcases.FIELD else 100)
    # CALLDATACOPY of a symbolic size, memory offset or calldata offset, and MLOAD /
    # MSTORE / MSTORE8 at symbolic offsets (environments.sol's batchTransfer moves
    # its free-memory pointer by a symbolic length) run on the device; what
    # escapes is the host's part
    # (memjump's jump to a target read back from symbolic memory is the host's by design)
    allowed = HOST_OPS | (WORLD_READS if name in symcases.FIELD else set()) | ({"JUMP"} if name == "memjump" else set()) \
        | ({"JUMPI"} if name == "balance_of" else set())      # the host-constant condition (see _min_forks)
    assert set(laser.escaped_ops) <= allowed, dict(laser.escaped_ops)


@pytest.mark.parametrize("name", symcases.SYM_CREATIONS_ALL)
def test_symbolic_creation_on_kernel1_equals_the_restatement(dev, name, monkeypatch):
    """transaction/symbolic.py's creation on kernel 1: the creation's calldata
    opcodes (CALLDATACOPY pops, CODESIZE + 0x200 with calldata.size pinned
    through an MG_REC_CDSIZE record, CODECOPY past the end of the code as a
    symbolic calldata copy) run on the device -- none of them escapes -- and
    every path ends as the restatement's does, constraint for constraint."""
    got, want, laser = symcases.run_creation_both(dev, name, monkeypatch)
    assert sum(want.values()) >= 2
    assert got == want, ([(k[:2], [str(c) for c in k[2]], v) for k, v in (got - want).items()],
                         [(k[:2], [str(c) for c in k[2]], v) for k, v in (want - got).items()])
    assert laser.lane_steps > (50 if name in symcases.SYM_CREATIONS else 10)
    for op in ("CODESIZE", "CODECOPY", "CALLDATACOPY", "CALLDATALOAD", "CALLDATASIZE"):
        assert laser.escaped_ops[op] == 0, (op, dict(laser.escaped_ops))
