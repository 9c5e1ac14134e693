"""Capacity escapes resumed inside their batch (LaserEVM._regrow_in_place) on
CPU with the oracle device.  A lane that fills its storage table or memory page
stops before the instruction with MG_ESCAPE; the batch is regrown 4x in that
capacity and the lane resumes where it stopped.  Every observable event (pre
hooks with their stacks, transaction ends, world-state adds) and the open
states must come out exactly as in a run whose capacities are large enough
from the start -- before round 2 the state restarted in a later batch and its
later events came after the batch's (known divergences)."""
import pytest

from mythril_amd.laser import (Account, BreadthFirstSearchStrategy, DepthFirstSearchStrategy,
                               Disassembly, LaserEVM, MessageCallTransaction, WorldState)
from mythril_amd.laser.transaction import _setup_global_state_for_execution
from mythril_amd import workloads
from oracle_device import OracleDevice

# i = 0; do { sstore(i, i); i += 1 } while (100 > i): 100 slots, the table starts at 64
STORE_LOOP = "60005b8080556001018060641160025700"
# mstore(0x2000, 1): past the 4 KiB page the batch starts with
MSTORE_FAR = "600161200052600051600055" + "00"
# two SSTOREs then a far MSTORE then an ADD: hooks on both sides of the escape
MIXED = "6001600155600260025560016130005260016002" + "0100"


def _txs(n_c2=24):
    b = workloads.c2_batch(n_c2, seed=5, stack_cap=64, mem_cap=1024)
    c2 = Disassembly(workloads.bytecode("overflow.sol.o"))
    odd = [STORE_LOOP, MSTORE_FAR, MIXED]
    out = []
    for i in range(n_c2):
        ws = WorldState()
        acct = Account(workloads.CONTRACT, code=c2)
        for k, val in b.storage_dict(i, drop_zero=False).items():
            acct.storage[k] = val
        ws.put_account(acct)
        out.append(MessageCallTransaction(
            world_state=ws, callee_account=acct, caller=workloads.ATTACKER,
            call_data=bytes(b.calldata[i, : int(b.calldata_len[i])]), gas_price=1,
            gas_limit=int(b.gas_limit[i]), origin=workloads.ATTACKER, call_value=0))
        if i % 4 == 1:
            dis = Disassembly(odd[(i // 4) % len(odd)])
            ws = WorldState()
            acct = Account(workloads.CONTRACT, code=dis)
            ws.put_account(acct)
            out.append(MessageCallTransaction(
                world_state=ws, callee_account=acct, caller=workloads.ATTACKER, call_data=b"",
                gas_price=1, gas_limit=8_000_000, origin=workloads.ATTACKER, call_value=0, code=dis))
    return out


def _run(strategy, grow, device=None):
    vm = LaserEVM(requires_statespace=False, device=device or OracleDevice(), strategy=strategy, execution_timeout=0)
    vm._cap_grow = grow
    log, tag = [], {}

    def who(state):
        return tag.get(id(state.current_transaction))

    def pre(name):
        def f(state):
            log.append(("pre", name, who(state), state.mstate.pc,
                        tuple(x.value for x in state.mstate.stack)))
        return f
    vm.register_hooks("pre", {op: [pre(op)] for op in ("SSTORE", "MSTORE", "ADD", "JUMPI", "STOP")})
    vm.register_laser_hooks("transaction_end",
                            lambda s, tx, ret, revert: log.append(("end", who(s), s.mstate.pc, revert)))
    vm.register_laser_hooks("add_world_state", lambda s: log.append(("ws", who(s))))
    for k, tx in enumerate(_txs()):
        _setup_global_state_for_execution(vm, tx)
        tag[id(tx)] = k
    vm.exec()
    opened = []
    for ws in vm.open_states:
        t = tag.get(id(ws.transaction_sequence[-1]))
        acct = ws.accounts[workloads.CONTRACT]
        opened.append((t, tuple(sorted((int(k), int(v)) for k, v in acct.storage.printable_storage.items()))))
    return log, opened, vm.regrows, vm.lane_steps


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_regrown_lanes_keep_the_event_order(strategy):
    log_big, open_big, regrows_big, steps_big = _run(strategy, 64)
    log, opened, regrows, steps = _run(strategy, 1)
    assert regrows_big == 0
    assert regrows >= 2                      # storage and memory escapes were resumed in place
    assert steps == steps_big
    assert len(log) == len(log_big) > 300
    assert log == log_big
    assert opened == open_big
    # the storage loop really wrote past the first table
    assert any(len(st) == 100 for _, st in opened)


def test_requeueing_instead_would_move_events(monkeypatch):
    """The batch above is not vacuous: restarting the escaped states in a later
    batch (the round-1 behaviour, still the fallback at a capacity limit)
    changes the BFS event log."""
    from mythril_amd.laser import svm as svm_mod
    log_big, open_big, _, _ = _run(BreadthFirstSearchStrategy, 64)
    monkeypatch.setattr(svm_mod.LaserEVM, "_regrow_in_place", lambda self, b, regrow, lanes: None)
    log, opened, regrows, _ = _run(BreadthFirstSearchStrategy, 1)
    assert regrows == 0
    assert log != log_big
