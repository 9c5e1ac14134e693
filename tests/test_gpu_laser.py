"""LaserEVM (mythril_amd.laser) on an MI355X: the reference's execution-loop API
driving kernel 1, checked against the reference harness and the oracle.

* VMTests through ``execute_message_call`` + ``LaserEVM.exec(track_gas=True)``,
  asserted exactly as tests/laser/evm_testsuite/evm_test.py:153-189 does;
* hooks: pre-hooks see the pre-state, post-hooks the successor, and both fire in
  the reference's BFS / DFS order — the expected sequence is derived by
  single-stepping the oracle;
* PluginSkipState / PluginSkipWorldState, coverage plugin, final states.
"""
import copy

import numpy as np
import pytest

from mythril_amd import workloads
from mythril_amd.device import GpuDevice
from mythril_amd.lanes import MG_ESCAPE, MG_RUNNING, LaneBatch, limbs_to_word
from mythril_amd.laser import (Account, BreadthFirstSearchStrategy, DepthFirstSearchStrategy,
                               Disassembly, InstructionCoveragePlugin, LaserEVM,
                               MessageCallTransaction, PluginSkipState, PluginSkipWorldState,
                               WorldState, execute_message_call)
from mythril_amd.laser.transaction import _setup_global_state_for_execution
from mythril_amd.smt.exponent_manager import exponent_function_manager
from mythril_amd.smt.expr import symbol_factory
from mythril_amd.smt.keccak_manager import keccak_function_manager
from oracle.evm_ref import OracleEVM
from vmtests_util import account, fill_lane, load_vmtests, vm_shape

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


# ------------------------------------------------------------------ VMTests
def _oracle_escapes(vectors):
    b = LaneBatch(vm_shape(vectors))
    o = OracleEVM()
    ids = {}
    for i, v in enumerate(vectors):
        if v["code"] not in ids:
            ids[v["code"]] = o.load_code(bytes.fromhex(v["code"]))
        fill_lane(b, i, v, ids[v["code"]])
    o.run(b)
    return {v["name"] for i, v in enumerate(vectors) if int(b.status[i]) == MG_ESCAPE}


def _run_vmtest(dev, v):
    """evm_test.py:124-152: the vector's pre-state, one concrete message call."""
    world_state = WorldState()
    for address, details in v["pre"].items():
        acct = Account(int(address, 16), concrete_storage=True)
        acct.code = Disassembly(details["code"])      # fixture codes carry no 0x
        acct.nonce = int(details["nonce"])
        for key, value in details["storage"].items():
            acct.storage[int(key, 16)] = int(value, 16)
        world_state.put_account(acct)
        acct.set_balance(int(details["balance"], 16))
    laser_evm = LaserEVM(requires_statespace=False, device=dev)
    laser_evm.open_states = [world_state]
    final_states = execute_message_call(
        laser_evm,
        callee_address=int(v["address"], 16),
        caller_address=int(v["caller"], 16),
        origin_address=int(v["origin"], 16),
        code=v["code"],
        gas_limit=int(v["gas"]),
        data=bytes.fromhex(v["data"]),
        gas_price=int(v["gas_price"], 16),
        value=int(v["value"], 16),
        track_gas=True,
    )
    return laser_evm, final_states


def test_vmtests_through_laser_evm(dev):
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    escaping = _oracle_escapes(vectors)
    passed = 0
    for v in vectors:
        if v["name"] in escaping:
            continue
        laser_evm, final_states = _run_vmtest(dev, v)
        gas_used = v["gas_used"]
        if gas_used is not None and gas_used < int(v["block_gas_limit"]):
            gas_min_max = [(s.mstate.min_gas_used, s.mstate.max_gas_used) for s in final_states]
            assert all(g[0] <= g[1] for g in gas_min_max), v["name"]
            assert any(g[0] <= gas_used for g in gas_min_max), v["name"]
        if v["post"] == {}:
            assert len(laser_evm.open_states) == 0, v["name"]
        else:
            assert len(laser_evm.open_states) == 1, v["name"]
            ws = laser_evm.open_states[0]
            for address, details in v["post"].items():
                acct = ws[int(address, 16)]
                assert acct.nonce == int(details["nonce"])
                assert acct.code.bytecode == details["code"]
                for index, value in details["storage"].items():
                    assert acct.storage[int(index, 16)].value == int(value, 16), v["name"]
        passed += 1
    assert passed == len(vectors) - len(escaping) == 499


# ------------------------------------------------------------------ function managers
def _oracle_records(vectors):
    shape = vm_shape(vectors)
    shape.rec_cap = 1 << 16
    b = LaneBatch(shape)
    o = OracleEVM()
    ids = {}
    for i, v in enumerate(vectors):
        if v["code"] not in ids:
            ids[v["code"]] = o.load_code(bytes.fromhex(v["code"]))
        fill_lane(b, i, v, ids[v["code"]])
    o.run(b)
    return [b.records(i) for i in range(b.n)]


def _hash_table():
    return [(k.value.to_bytes(k.size() // 8, "big"), h.value)
            for k, h in keccak_function_manager.concrete_hashes.items()]


def test_vmtests_function_manager_registrations(dev):
    """Every SHA3 of a concrete slice lands in keccak_function_manager.concrete_hashes
    and every concrete EXP adds result == Power(base, exp) to the path's
    constraints, as the oracle's records of the same vectors say."""
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    escaping = _oracle_escapes(vectors)
    records = _oracle_records(vectors)
    checked = 0
    for v, recs in zip(vectors, records):
        if v["name"] in escaping or not recs:
            continue
        keccak_function_manager.reset()
        _, final_states = _run_vmtest(dev, v)
        want = []
        for r in recs:
            if r[1] == "keccak" and (r[2], r[3]) not in want:
                want.append((r[2], r[3]))
        assert _hash_table() == want, v["name"]
        want_c = [exponent_function_manager.create_condition(
            symbol_factory.BitVecVal(r[2], 256), symbol_factory.BitVecVal(r[3], 256))[1].raw
            for r in recs if r[1] == "exp"]
        assert final_states, v["name"]
        for s in final_states:
            # after the transaction's UGE(balances[caller], value) conjunct
            # (transaction_models.py:127-148)
            assert [c.raw for c in s.world_state.constraints][1:] == want_c, v["name"]
        checked += 1
    keccak_function_manager.reset()
    assert checked >= 15


# ------------------------------------------------------------------ hooks
CODE = workloads.bytecode("overflow.sol.o")


def _c2_states(n, seed=5):
    """n message calls of the C2 workload as GlobalStates (one world state each)."""
    b = workloads.c2_batch(n, seed=seed, stack_cap=64, mem_cap=1024)
    states = []
    for i in range(n):
        ws = WorldState()
        acct = Account(workloads.CONTRACT, code=Disassembly(CODE))
        for k, val in b.storage_dict(i, drop_zero=False).items():
            acct.storage[k] = val
        ws.put_account(acct)
        tx = MessageCallTransaction(
            world_state=ws, callee_account=acct, caller=workloads.ATTACKER,
            call_data=bytes(b.calldata[i, : int(b.calldata_len[i])]), gas_price=1,
            gas_limit=int(b.gas_limit[i]), origin=workloads.ATTACKER, call_value=0)
        states.append(tx)
    return b, states


def _oracle_events(b, pre_ops, post_ops):
    """Single-step every lane on the oracle; return per lane the sequence of
    (kind, round, pc, stack) a pre hook on `pre_ops` / post hook on `post_ops`
    would observe."""
    o = OracleEVM()
    cid = o.load_code(CODE)
    ref = b.copy()
    ref.code_id[:] = cid
    ops, _ = o.code_table(cid)
    events = {i: [] for i in range(b.n)}
    pending_post = {}
    for rnd in range(100000):
        live = [i for i in range(b.n) if int(ref.status[i]) == MG_RUNNING]
        if not live:
            break
        for i in live:
            if i in pending_post:
                events[i].append(("post", pending_post.pop(i), int(ref.pc[i]),
                                  tuple(ref.stack_words(i))))
            pc = int(ref.pc[i])
            if pc < ops.size and int(ops[pc]) in pre_ops:
                events[i].append(("pre", rnd, pc, tuple(ref.stack_words(i))))
        before = {i: int(ref.pc[i]) for i in live}
        o.run(ref, max_steps=1)
        for i in live:
            pc = before[i]
            if pc < ops.size and int(ops[pc]) in post_ops and int(ref.status[i]) == MG_RUNNING:
                pending_post[i] = rnd
    return events


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_hooks_fire_in_reference_order(dev, strategy):
    n = 96
    b, txs = _c2_states(n)
    pre_ops, post_ops = {0x55, 0x57}, {0x54}        # SSTORE, JUMPI pre; SLOAD post
    expected = _oracle_events(b, pre_ops, post_ops)
    vm = LaserEVM(requires_statespace=False, device=dev, strategy=strategy)
    log = []
    pos = {}

    def rec(kind):
        def f(state):
            log.append((kind, pos[id(state.current_transaction)],
                        state.mstate.pc, tuple(x.value for x in state.mstate.stack)))
        return f

    vm.register_hooks("pre", {"SSTORE": [rec("pre")], "JUMPI": [rec("pre")]})
    vm.register_hooks("post", {"SLOAD": [rec("post")]})
    for i, tx in enumerate(txs):
        _setup_global_state_for_execution(vm, tx)
        pos[id(tx)] = i            # hooked states are the hooks' own: a path is its transaction
    vm.exec()
    # expected global order from per-lane sequences
    flat = [(k, r, i, pc, st) for i, evs in expected.items() for (k, r, pc, st) in evs]
    if strategy is BreadthFirstSearchStrategy:
        flat.sort(key=lambda e: (e[1], e[2], e[0] == "pre"))
    else:
        flat.sort(key=lambda e: (-e[2], e[1], e[0] == "pre"))
    want = [(k, i, pc, st) for (k, r, i, pc, st) in flat]
    assert len(log) == len(want) > n
    assert log == want


def test_skip_state_and_skip_world_state(dev):
    n = 64
    b, txs = _c2_states(n, seed=9)
    # reference: lanes reaching SSTORE are dropped by the pre hook
    o = OracleEVM()
    ref = b.copy()
    ref.code_id[:] = o.load_code(CODE)
    o.run(ref, hook_mask=(0, 1 << 0x15, 0, 0))        # stop before SSTORE (0x55 = 64+21)
    reaching = {i for i in range(n) if int(ref.status[i]) == 7}
    assert 0 < len(reaching) < n

    vm = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy)

    def skip(state):
        raise PluginSkipState

    vm.register_hooks("pre", {"SSTORE": [skip]})
    for tx in txs:
        _setup_global_state_for_execution(vm, tx)
    final = vm.exec(track_gas=True)
    o2 = OracleEVM()
    full = b.copy()
    full.code_id[:] = o2.load_code(CODE)
    o2.run(full)
    kept = [i for i in range(n) if i not in reaching and int(full.status[i]) in (1, 2, 4)]
    assert len(vm.open_states) == len(kept)
    assert len(final) == n      # skipped states have no successor: final (svm.py:328-334)

    vm2 = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy)

    @vm2.laser_hook("add_world_state")
    def no_world(state):
        raise PluginSkipWorldState

    _, txs2 = _c2_states(n, seed=9)
    for tx in txs2:
        _setup_global_state_for_execution(vm2, tx)
    vm2.exec()
    assert vm2.open_states == []


def test_final_states_and_storage_match_oracle(dev):
    n = 200
    b, txs = _c2_states(n, seed=21)
    o = OracleEVM()
    ref = b.copy()
    ref.code_id[:] = o.load_code(CODE)
    o.run(ref)
    vm = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy)
    for tx in txs:
        _setup_global_state_for_execution(vm, tx)
    states = list(vm.work_list)
    final = vm.exec(track_gas=True)
    assert {id(s) for s in final} == {id(s) for s in states}
    # BFS: final states ordered by (halting round, position)
    idx = {id(s): i for i, s in enumerate(states)}
    rounds = [int(ref.steps[i]) - 1 for i in range(n)]
    assert [idx[id(s)] for s in final] == sorted(range(n), key=lambda i: (rounds[i], i))
    for s in final:
        i = idx[id(s)]
        assert s.mstate.pc == int(ref.pc[i])
        assert (s.mstate.min_gas_used, s.mstate.max_gas_used) == (int(ref.gas_min[i]),
                                                                  int(ref.gas_max[i]))
        assert [x.value for x in s.mstate.stack] == ref.stack_words(i)
        assert s.environment.active_account.storage.printable_storage == ref.storage_dict(
            i, drop_zero=False)
    assert vm.lane_steps == int(ref.steps.sum())


def test_coverage_plugin_matches_oracle(dev):
    n = 128
    b, txs = _c2_states(n, seed=33)
    o = OracleEVM()
    cid = o.load_code(CODE)
    ops, _ = o.code_table(cid)
    ref = b.copy()
    ref.code_id[:] = cid
    covered = np.zeros(ops.size, dtype=bool)
    for _ in range(100000):
        live = [i for i in range(n) if int(ref.status[i]) == MG_RUNNING]
        if not live:
            break
        for i in live:
            if int(ref.pc[i]) < ops.size:
                covered[int(ref.pc[i])] = True
        o.run(ref, max_steps=1)
    vm = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy)
    plugin = InstructionCoveragePlugin()
    plugin.initialize(vm)
    dev.coverage_clear()
    for tx in txs:
        _setup_global_state_for_execution(vm, tx)
    vm.exec()
    (nins, bits), = [v for k, v in plugin.coverage.items()]
    assert nins == ops.size
    assert bits == covered.tolist()


# ------------------------------------------------------------ BoundedLoopsStrategy
def _loop_states(vm, ns):
    from test_loop_bound import LOOP
    for n in ns:
        ws = WorldState()
        acct = Account(0xC0DE, code=Disassembly(LOOP))
        ws.put_account(acct)
        tx = MessageCallTransaction(world_state=ws, callee_account=acct, caller=0xCA11,
                                    call_data=int(n).to_bytes(32, "big"), gas_price=1,
                                    gas_limit=10 ** 7, origin=0xCA11, call_value=0)
        _setup_global_state_for_execution(vm, tx)
    return list(vm.work_list)


@pytest.mark.parametrize("hooked", [False, True])
def test_bounded_loops_strategy_drops_like_the_oracle(dev, hooked):
    from mythril_amd.laser import BoundedLoopsStrategy, JumpdestCountAnnotation
    from test_loop_bound import LOOP, loop_batch
    ns = list(range(0, 12)) + [50, 2 ** 100]
    b = loop_batch(ns)
    o = OracleEVM()
    b.code_id[:] = o.load_code(LOOP)
    o.run(b, loop_bound=3)
    vm = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy)
    vm.extend_strategy(BoundedLoopsStrategy, loop_bound=3)
    seen = []
    if hooked:
        vm.register_hooks("pre", {"JUMPDEST": [lambda s: seen.append(s.mstate.pc)]})
    states = _loop_states(vm, ns)
    final = vm.exec(track_gas=True)
    halted = [i for i in range(len(ns)) if int(b.status[i]) == 1]
    assert len(vm.open_states) == len(halted)
    # a hooked state stays the hooks' own and its path goes on with a copy (as in
    # the reference): paths are told apart by their transaction
    by_tx = {id(s.current_transaction): s for s in final}
    assert set(by_tx) == {id(states[i].current_transaction) for i in halted}
    for i in halted:
        ann = [a for a in by_tx[id(states[i].current_transaction)].annotations
               if isinstance(a, JumpdestCountAnnotation)]
        assert ann and ann[0].trace == [int(x) for x in b.trace[i, : int(b.trace_len[i])]]
    if hooked:
        # every JUMPDEST pop that survived the bound fired the hook once
        assert len(seen) == sum(1 for i in range(len(ns))
                                for x in b.trace[i, : int(b.trace_len[i])] if x == 3) \
            - sum(1 for i in range(len(ns)) if int(b.status[i]) == 10)


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_keccak_registrations_in_reference_order(dev, strategy):
    """C2 paths hash mapping slots.  The reference registers each concrete hash
    when its SHA3 executes, so a hook sees exactly the hashes of instructions
    that ran before it in the strategy's global order; the final table holds
    them in first-execution order."""
    n = 96
    _, txs = _c2_states(n)
    b = workloads.c2_batch(n, seed=5, stack_cap=64, mem_cap=1024, rec_cap=512)
    events = _oracle_events(b.copy(), {0x55}, set())
    o = OracleEVM()
    b.code_id[:] = o.load_code(CODE)
    o.run(b)
    bfs = strategy is BreadthFirstSearchStrategy
    key = (lambda step, i: (step, i)) if bfs else (lambda step, i: (-i, step))
    recs = sorted((key(r[0], i), r[2], r[3]) for i in range(n) for r in b.records(i)
                  if r[1] == "keccak")
    assert len(recs) > n

    def seen_before(k):
        out = []
        for rk, data, h in recs:
            if rk < k and (data, h) not in out:
                out.append((data, h))
        return len(out)

    flat = sorted((key(rnd, i), i) for i, evs in events.items() for (_, rnd, _, _) in evs)
    want = [seen_before(k) for k, _ in flat]
    keccak_function_manager.reset()
    vm = LaserEVM(requires_statespace=False, device=dev, strategy=strategy)
    log = []
    vm.register_hooks("pre", {"SSTORE": [lambda s: log.append(len(keccak_function_manager.concrete_hashes))]})
    for tx in txs:
        _setup_global_state_for_execution(vm, tx)
    vm.exec()
    assert len(log) == len(want) > 0
    assert log == want
    final = []
    for _, data, h in recs:
        if (data, h) not in final:
            final.append((data, h))
    assert _hash_table() == final
    keccak_function_manager.reset()


# ------------------------------------------------------------------ sharded transaction rounds
def test_transaction_rounds_device_equal_oracle_device(dev):
    """laser/sharded.py's rounds (one rank) on kernel 1 give the same open world
    states, coverage and transaction ids as on the oracle-backed device that the
    multi-rank gloo tests (test_sharded_cpu.py) use."""
    import test_sharded_cpu as ts
    from mythril_amd.laser import (Account, InstructionCoveragePlugin, WorldState,
                                   tx_id_manager)
    from mythril_amd.laser.sharded import execute_message_calls
    from mythril_amd import workloads

    tx_id_manager.restart_counter()
    ws = WorldState()
    acct = Account(ts.CALLEE, concrete_storage=True)
    acct.code = Disassembly(workloads.bytecode("overflow.sol.o").hex())
    ws.put_account(acct)
    vm = LaserEVM(requires_statespace=False, device=dev)
    cov = InstructionCoveragePlugin()
    cov.initialize(vm)
    vm.open_states = [ws]
    ids = []
    for _ in range(ts.ROUNDS):
        execute_message_calls(vm, ts.CALLEE, ts.ATTACKER, ts.ATTACKER, ts.DATAS,
                              gas_limit=8_000_000, gas_price=0, value=0)
        ids.extend(s.transaction_sequence[-1].id for s in vm.open_states)
    prints = sorted((tuple(sorted(s[ts.CALLEE].storage.items())), str(s[ts.CALLEE].balance().raw))
                    for s in vm.open_states)
    table = {k: list(v[1]) for k, v in vm.coverage().items()}
    ref = ts._rounds()
    assert prints == ref[0]
    assert table == ref[1]
    assert tx_id_manager._next_transaction_id == ref[2]
    assert ids == ref[3]
    assert vm.lane_steps == ref[4]
