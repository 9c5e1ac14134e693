"""BoundedLoopsStrategy and a past-the-end pc (strategy/extensions/bounded_loops.py:103-145):
the strategy reads the popped state's current instruction, the IndexError of a
pc past the end becomes StopIteration and ends the whole exec.  The batched
LaserEVM stops at that event in the reference's BFS order: states whose events
come earlier are processed, the rest of the work list is abandoned."""
from mythril_amd import workloads
from mythril_amd.laser import (Account, BoundedLoopsStrategy, BreadthFirstSearchStrategy, Disassembly,
                               LaserEVM, MessageCallTransaction, WorldState)
from mythril_amd.laser.transaction import _setup_global_state_for_execution
from oracle_device import OracleDevice

SHORT = "6001"                  # PUSH1 1, then past the end at round 1
LONG = "600160016001600100"     # 4 x PUSH1, STOP at round 4


def _run(codes, bounded):
    vm = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=BreadthFirstSearchStrategy, execution_timeout=0)
    if bounded:
        vm.extend_strategy(BoundedLoopsStrategy, loop_bound=3)
    ends = []
    vm.register_laser_hooks("transaction_end", lambda s, tx, r, rev: ends.append(s.environment.code.bytecode))
    for code in codes:
        ws = WorldState()
        acct = Account(workloads.CONTRACT, code=Disassembly(code))
        ws.put_account(acct)
        _setup_global_state_for_execution(vm, MessageCallTransaction(
            world_state=ws, callee_account=acct, caller=workloads.ATTACKER, call_data=b"",
            gas_limit=8_000_000, origin=workloads.ATTACKER, code=Disassembly(code)))
    vm.exec()
    return len(vm.open_states), ends


def test_past_the_end_pop_ends_exec_under_bounded_loops():
    # without the extension both paths end normally (END adds its world state)
    assert _run([SHORT, LONG], bounded=False)[0] == 2
    # with it, the SHORT path's pop at round 1 ends exec before LONG reaches STOP
    n, ends = _run([SHORT, LONG], bounded=True)
    assert n == 0 and ends == []
    # a path that ends (STOP) before the cut is processed
    n, ends = _run(["00", "6001600160016001"], bounded=True)
    assert n == 1 and len(ends) == 1
