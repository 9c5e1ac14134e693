"""Hook batching of the BFS event loop (LaserEVM._ack_safe) on CPU with the
oracle device: deferring the launch that executes a resumed hooked instruction
to the end of its round must leave every observable event exactly where the
one-launch-per-event loop puts it (that loop is pinned against single-stepped
oracle runs by test_gpu_laser.py::test_hooks_fire_in_reference_order).

The batch mixes C2 lanes with lanes whose hooked instruction ends or escapes
the path at its own round -- the cases _ack_safe must refuse: invalid JUMP,
JUMPI to a bad target (dropped), a real stack underflow behind the table's
precheck (DUP3), OOG on a hooked ADD, an MSTORE past the lane's memory page,
STOP/RETURN/REVERT."""
import pytest

import bench
from mythril_amd import workloads
from mythril_amd.laser import (Account, BreadthFirstSearchStrategy, DepthFirstSearchStrategy,
                               Disassembly, LaserEVM, MessageCallTransaction, WorldState)
from mythril_amd.laser import svm as svm_mod
from mythril_amd.laser.transaction import _setup_global_state_for_execution
from oracle_device import OracleDevice

ODD_CODES = [
    ("6001600201600556", 8_000_000),          # ADD, JUMP to 5 (not a JUMPDEST): VmException
    ("6001602057", 8_000_000),                # JUMPI to 0x20 (past the end): dropped
    ("600160028200", 8_000_000),              # DUP3 with two words: real underflow
    ("6001600201600201", 8),                  # the first ADD runs out of gas (limit 8)
    ("6001620100005200", 8_000_000),          # MSTORE at 0x10000: past the memory page
    ("600160025b01600456", 8_000_000),         # a JUMP back to the JUMPDEST: ADD then underflow
    ("600160005260206000f3", 8_000_000),      # MSTORE, RETURN
    ("60006000fd", 8_000_000),                # REVERT
]


def _states(n_c2=48):
    b = workloads.c2_batch(n_c2, seed=21, stack_cap=64, mem_cap=1024)
    code = Disassembly(workloads.bytecode("overflow.sol.o"))
    txs = []
    for i in range(n_c2):
        ws = WorldState()
        acct = Account(workloads.CONTRACT, code=code)
        for k, val in b.storage_dict(i, drop_zero=False).items():
            acct.storage[k] = val
        ws.put_account(acct)
        txs.append(MessageCallTransaction(
            world_state=ws, callee_account=acct, caller=workloads.ATTACKER,
            call_data=bytes(b.calldata[i, : int(b.calldata_len[i])]), gas_price=1,
            gas_limit=int(b.gas_limit[i]), origin=workloads.ATTACKER, call_value=0))
        if i % 6 == 3:                        # odd lanes interleaved with the C2 lanes
            hexcode, gas = ODD_CODES[(i // 6) % len(ODD_CODES)]
            ws = WorldState()
            dis = Disassembly(hexcode)
            acct = Account(workloads.CONTRACT, code=dis)
            ws.put_account(acct)
            txs.append(MessageCallTransaction(
                world_state=ws, callee_account=acct, caller=workloads.ATTACKER, call_data=b"",
                gas_price=1, gas_limit=gas, origin=workloads.ATTACKER, call_value=0, code=dis))
    return txs


def _run(strategy, batching, monkeypatch):
    if batching is False:
        monkeypatch.setattr(svm_mod.LaserEVM, "_ack_safe", lambda self, name, s, b: False)
    elif batching:
        monkeypatch.undo()
    vm = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=strategy, execution_timeout=0)
    log = []
    tag = {}

    def who(state):
        # a hooked state is the hooks' own (the lane goes on with a copy, as the
        # reference's evaluate does): paths are told apart by their transaction
        return tag.get(id(state.current_transaction))

    def pre(name):
        def f(state):
            log.append(("pre", name, who(state), state.mstate.pc,
                        tuple(x.value for x in state.mstate.stack)))
        return f
    vm.register_hooks("pre", {op: [pre(op)] for op in bench.DEFAULT_MODULE_PRE + ["DUP3", "SWAP1"]})
    vm.register_laser_hooks("transaction_end",
                            lambda s, tx, ret, revert: log.append(("end", who(s), s.mstate.pc, revert)))
    vm.register_laser_hooks("add_world_state", lambda s: log.append(("ws", who(s))))
    for k, tx in enumerate(_states()):
        _setup_global_state_for_execution(vm, tx)
        tag[id(tx)] = k
    vm.exec()
    opened = [tag.get(id(ws.transaction_sequence[-1])) for ws in vm.open_states]
    return log, opened, vm.launches, vm.lane_steps


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_batched_hook_rounds_keep_the_event_order(strategy, monkeypatch):
    log0, open0, launches0, steps0 = _run(strategy, False, monkeypatch)
    log1, open1, launches1, steps1 = _run(strategy, True, monkeypatch)
    assert steps1 == steps0
    assert len(log1) == len(log0) > 500
    assert log1 == log0
    assert open1 == open0
    kinds = {e[0] for e in log0}
    assert {"pre", "end", "ws"} <= kinds
    if strategy is BreadthFirstSearchStrategy:
        assert launches1 * 3 < launches0          # rounds share launches
    else:
        assert launches1 == launches0             # DFS: unchanged


@pytest.mark.parametrize("unguarded", ["DUP3", "ADD"])
def test_the_batch_exercises_the_guards(unguarded, monkeypatch):
    """Deferring `unguarded` without _ack_safe's checks (stack underflow behind
    DUP3's precheck, OOG on ADD) would move an event: the batch above reaches
    those cases, so its equality is not vacuous."""
    log0, open0, _, _ = _run(BreadthFirstSearchStrategy, False, monkeypatch)
    monkeypatch.undo()
    orig = svm_mod.LaserEVM._ack_safe
    monkeypatch.setattr(svm_mod.LaserEVM, "_ack_safe",
                        lambda self, name, s, b: True if name == unguarded else orig(self, name, s, b))
    log2, open2, _, _ = _run(BreadthFirstSearchStrategy, None, _NoUndo())
    assert (log2, open2) != (log0, open0)


class _NoUndo:
    def undo(self):
        pass


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_host_halts_equal_device_halts(strategy, monkeypatch):
    """LaserEVM._halts_on_host ends a hooked STOP / RETURN on the host instead of
    launching the device to report it: the event log, open states and lane-steps
    must be those of the device run (the batch includes RETURNs of in-memory data
    and the odd codes' halts)."""
    log_h, open_h, launches_h, steps_h = _run(strategy, True, monkeypatch)
    monkeypatch.setattr(svm_mod.LaserEVM, "_halts_on_host", lambda self, name, s, b, i: False)
    log_d, open_d, launches_d, steps_d = _run(strategy, None, _NoUndo())
    assert steps_h == steps_d
    assert log_h == log_d
    assert open_h == open_d
    assert launches_h < launches_d


@pytest.mark.parametrize("keep", ["state", "mstate", "world_state", "storage", "nothing"])
def test_a_kept_state_stays_the_one_the_hook_saw(keep, monkeypatch):
    """The lane goes on with the hooked state itself when no hook kept it or a
    part of it the lane changes later (svm._held); a hook that keeps the state
    (or its machine state, world state or storage) must find it exactly as it
    saw it after exec, as with the reference's copy per evaluate
    (instructions.py:121-130) -- and the event log must not depend on it."""
    vm = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=BreadthFirstSearchStrategy, execution_timeout=0)
    kept, seen, log = [], [], []

    def part(state):
        return {"state": state, "mstate": state.mstate, "world_state": state.world_state,
                "storage": state.environment.active_account.storage, "nothing": None}[keep]

    def view(state):
        st = state.environment.active_account.storage
        return (state.mstate.pc, tuple(x.value for x in state.mstate.stack), state.mstate.min_gas_used,
                len(state.world_state.constraints), tuple(sorted(st.printable_storage.items())))

    def hook(state):
        log.append(view(state))
        p = part(state)
        if p is not None and len(kept) < 400:
            kept.append(p)
            seen.append(view(state))
    vm.register_hooks("pre", {op: [hook] for op in ("ADD", "SSTORE", "SLOAD", "JUMPI", "MSTORE")})
    for tx in _states(24):
        _setup_global_state_for_execution(vm, tx)
    vm.exec()
    if keep != "nothing":
        assert len(kept) > 50
    for k, obj in enumerate(kept):
        if keep == "state":
            assert view(obj) == seen[k]
        elif keep == "mstate":
            assert (obj.pc, tuple(x.value for x in obj.stack), obj.min_gas_used) == seen[k][:3]
        elif keep == "world_state":
            st = obj[workloads.CONTRACT].storage
            assert (len(obj.constraints), tuple(sorted(st.printable_storage.items()))) == seen[k][3:]
        else:
            assert tuple(sorted(obj.printable_storage.items())) == seen[k][4]
    ref = _log_without_keeping()
    assert log == ref


def _log_without_keeping():
    vm = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=BreadthFirstSearchStrategy, execution_timeout=0)
    log = []

    def hook(state):
        st = state.environment.active_account.storage
        log.append((state.mstate.pc, tuple(x.value for x in state.mstate.stack), state.mstate.min_gas_used,
                    len(state.world_state.constraints), tuple(sorted(st.printable_storage.items()))))
    vm.register_hooks("pre", {op: [hook] for op in ("ADD", "SSTORE", "SLOAD", "JUMPI", "MSTORE")})
    for tx in _states(24):
        _setup_global_state_for_execution(vm, tx)
    vm.exec()
    return log


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_plain_hook_fast_path_equals_the_general_path(strategy, monkeypatch):
    """LaserEVM._deliver_plain_hook (plain lanes, pre hooks only) against the
    general MG_HOOK branch, with hooks that leave the state alone, rewrite a
    stack word, write memory, write storage, and keep the state: the same event
    log, open states and lane-steps."""
    def run(fast):
        monkeypatch.setattr(svm_mod.LaserEVM, "_fast_hooks", fast)
        vm = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=strategy, execution_timeout=0)
        log, kept = [], []

        def view(state):
            st = state.environment.active_account.storage
            return (state.mstate.pc, tuple(x.value for x in state.mstate.stack), state.mstate.min_gas_used,
                    bytes(state.mstate.memory.raw()), tuple(sorted(st.printable_storage.items())))

        def on_add(state):
            log.append(("ADD",) + view(state))
            if state.mstate.pc % 3 == 0:
                state.mstate.stack[-1] = state.mstate.stack[-1] + 1      # rewrite an operand

        def on_mstore(state):
            log.append(("MSTORE",) + view(state))
            if len(state.mstate.memory) >= 32 and state.mstate.pc % 2:
                state.mstate.memory[5] = 0x42                              # write memory

        def on_sload(state):
            log.append(("SLOAD",) + view(state))
            state.environment.active_account.storage[0x99] = 7              # write storage

        def on_jumpi(state):
            log.append(("JUMPI",) + view(state))
            if len(kept) < 50:
                kept.append(state)
        vm.register_hooks("pre", {"ADD": [on_add], "MSTORE": [on_mstore], "SLOAD": [on_sload],
                                  "JUMPI": [on_jumpi], "SSTORE": [lambda st: log.append(("SSTORE",) + view(st))]})
        vm.register_laser_hooks("transaction_end", lambda st, tx, ret, revert: log.append(("end", revert) + view(st)))
        for tx in _states(30):
            _setup_global_state_for_execution(vm, tx)
        vm.exec()
        return log, [view(k) for k in kept], sorted(view(w) for w in
                                                   [s for s in vm.open_states] if hasattr(w, "mstate")), vm.lane_steps
    fast = run(True)
    slow = run(False)
    assert fast == slow
    assert len(fast[0]) > 300


@pytest.mark.parametrize("fast", [True, False])
def test_hooks_that_keep_nothing_cost_no_state_copy(fast, monkeypatch):
    """A pre hook that keeps no reference lets the lane go on with the hooked
    state itself (no GlobalState copy per event), on the fast path and on the
    general branch; a hook that keeps the state gets one copy per event."""
    from mythril_amd.laser import state as state_mod
    monkeypatch.setattr(svm_mod.LaserEVM, "_fast_hooks", fast)
    copies = [0]
    orig = state_mod.GlobalState.__copy__

    def counting(self):
        copies[0] += 1
        return orig(self)
    monkeypatch.setattr(state_mod.GlobalState, "__copy__", counting)
    for keep, want_copies in ((False, False), (True, True)):
        copies[0] = 0
        kept, events = [], [0]
        vm = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=BreadthFirstSearchStrategy, execution_timeout=0)

        def hook(st):
            events[0] += 1
            if keep:
                kept.append(st)
        vm.register_hooks("pre", {op: [hook] for op in ("ADD", "SLOAD", "JUMPI", "MSTORE")})
        for tx in _states(12):
            _setup_global_state_for_execution(vm, tx)
        vm.exec()
        assert events[0] > 100
        assert (copies[0] >= events[0]) if want_copies else copies[0] == 0, (keep, copies[0], events[0])
