"""Taint lanes on CPU (oracle device + tests/taintref.py as the taint stepper):
the integer module's ADD/SUB/MUL/EXP annotations and SSTORE/JUMPI collections
and TxOrigin's ORIGIN annotation, run as device actions (laser/taint.py
BATCH_SAFE), must leave the same annotations, state annotations and issues as
running every hook on the host -- and as a run where every opcode is a host
event, the closest the mirror gets to the reference's one-state-per-step loop.
The modules are the restatements in tests/refmodules.py (the reference's cannot
be imported here); parity with the reference itself is unpinned (no z3)."""
import pytest

from mythril_amd import workloads
from mythril_amd.laser import (Account, BreadthFirstSearchStrategy, DepthFirstSearchStrategy, Disassembly,
                               LaserEVM, MessageCallTransaction, WorldState)
from mythril_amd.laser import taint as tnt
from mythril_amd.laser.opcodes import OPCODES
from mythril_amd.laser.transaction import _setup_global_state_for_execution
from oracle_device import OracleDevice
import refmodules
from refmodules import IntegerArithmetics, OverUnderflowStateAnnotation, TxOrigin, hooks_of

DEFAULT_SET = ("IntegerArithmetics", "TxOrigin", "ArbitraryStorage", "ArbitraryJump", "UserAssertions",
               "Exceptions", "StateChangeAfterCall")


def _txs(n_c2=24, n_under=8, n_origin=8, extra=()):
    out = []
    b = workloads.c2_batch(n_c2, seed=33, stack_cap=64, mem_cap=1024)
    code = Disassembly(workloads.bytecode("overflow.sol.o"))
    for i in range(n_c2):
        ws = WorldState()
        acct = Account(workloads.CONTRACT, code=code)
        for k, val in b.storage_dict(i, drop_zero=False).items():
            acct.storage[k] = val
        ws.put_account(acct)
        out.append(MessageCallTransaction(
            world_state=ws, callee_account=acct, caller=workloads.ATTACKER,
            call_data=bytes(b.calldata[i, : int(b.calldata_len[i])]), gas_price=1,
            gas_limit=int(b.gas_limit[i]), origin=workloads.ATTACKER, call_value=0))
    import random
    rnd = random.Random(7)
    for name, n in (("underflow.sol.o", n_under), ("origin.sol.o", n_origin)) + tuple(extra):
        dis = Disassembly(workloads.bytecode(name))
        sels = sorted({ins["argument"] for ins in dis.instruction_list
                       if ins["opcode"] == "PUSH4" and isinstance(ins.get("argument"), str)})
        for k in range(n):
            ws = WorldState()
            acct = Account(workloads.CONTRACT, code=dis)
            acct.storage[0] = rnd.getrandbits(256)
            acct.storage[1] = rnd.getrandbits(16)
            ws.put_account(acct)
            sel = bytes.fromhex(sels[k % len(sels)][2:].rjust(8, "0")) if sels else b""
            cd = sel + rnd.getrandbits(160).to_bytes(32, "big") + rnd.getrandbits(256).to_bytes(32, "big")
            origin = workloads.ATTACKER if k % 2 else 0xAFFE
            out.append(MessageCallTransaction(
                world_state=ws, callee_account=acct, caller=origin, call_data=cd, gas_price=1,
                gas_limit=8_000_000, origin=origin, call_value=0, code=dis))
    return out


def _run(strategy, mode, monkeypatch, device=None, modules=("IntegerArithmetics", "TxOrigin"), extra=()):
    """mode: "device" (batch-safe hooks as device actions), "host" (every module
    hook on the host), "every" (every opcode a host event)."""
    monkeypatch.undo()
    if mode != "device":
        monkeypatch.setattr(tnt, "BATCH_SAFE", {})
    # the modules confirm issues through the SAT-only backend (as tests/analyze.py):
    # the concrete paths' constant sets are decided directly, the EXP points'
    # Power(b, e) == r conjuncts by the search's axiom completion
    from mythril_amd.smt import solver
    from mythril_amd.smt.search import SatSearchBackend
    from oracle_device import OracleK2
    mc = solver.ModelCache(device=device or OracleK2())
    monkeypatch.setattr(solver, "model_cache", mc)
    monkeypatch.setattr(solver, "solver_backend", SatSearchBackend(mc))
    solver.get_model.cache_clear()
    vm = LaserEVM(requires_statespace=False, device=device or OracleDevice(), strategy=strategy, execution_timeout=0)
    vm.track_objects = True
    mods = [getattr(refmodules, m)() for m in modules]
    vm.register_hooks("pre", hooks_of(mods, "pre"))
    vm.register_hooks("post", hooks_of(mods, "post"))
    if mode == "every":
        vm.register_hooks("pre", {op: [lambda s: None] for op in OPCODES})
    tag, ends = {}, []

    def end(state, tx, ret, revert):
        sa = [a for a in state.annotations if isinstance(a, OverUnderflowStateAnnotation)]
        got = sorted((a.operator, a.overflowing_state.get_current_instruction()["address"],
                      a.constraint.value) for s in sa for a in s.overflowing_state_annotations)
        stack = [sorted((type(a).__name__, getattr(a, "operator", "")) for a in x.annotations)
                 for x in state.mstate.stack]
        # an empty PotentialIssuesAnnotation (StateChangeAfterCall's SLOAD / SSTORE
        # hook adds one even when it files nothing) is left out: the device skips
        # that hook without a state annotation, and nothing reads an empty one
        # (check_potential_issues makes its own, beam search weighs it 0)
        pots = [tuple(p.potential_issues) for p in state.annotations
                if isinstance(p, refmodules.PotentialIssuesAnnotation) and p.potential_issues]
        jumps = [a.last_jump for a in state.annotations if isinstance(a, refmodules.LastJumpAnnotation)]
        ends.append((tag[id(tx)], state.mstate.pc, revert, bool(sa), tuple(got), str(stack), str(pots),
                     tuple(jumps)))
    vm.register_laser_hooks("transaction_end", end)
    for k, tx in enumerate(_txs(extra=extra)):
        _setup_global_state_for_execution(vm, tx)
        tag[id(tx)] = k
    vm.exec()
    issues = sorted(i.key() for m in mods for i in m.issues)
    return sorted(ends), issues, vm.launches, vm.lane_steps


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_device_taint_matches_host_hooks(strategy, monkeypatch):
    ends_d, issues_d, launches_d, steps_d = _run(strategy, "device", monkeypatch)
    ends_h, issues_h, launches_h, steps_h = _run(strategy, "host", monkeypatch)
    assert steps_d == steps_h
    assert ends_d == ends_h
    assert issues_d == issues_h
    # not vacuous: integer issues (sendeth's underflow on overflow.sol.o) and
    # collected state annotations exist, and the device spared host events
    assert any(i[0] == "101" for i in issues_d)
    assert sum(1 for e in ends_d if e[4]) > 5
    assert launches_d < launches_h


def test_device_taint_matches_every_opcode_on_the_host(monkeypatch):
    ends_d, issues_d, _, steps_d = _run(BreadthFirstSearchStrategy, "device", monkeypatch)
    ends_e, issues_e, _, steps_e = _run(BreadthFirstSearchStrategy, "every", monkeypatch)
    assert steps_d == steps_e
    assert ends_d == ends_e
    assert issues_d == issues_e


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_default_module_set_on_the_device_matches_host_hooks(strategy, monkeypatch):
    """The wider set (deferred potential issues of ArbitraryStorage, the
    LastJumpAnnotation of Exceptions, UserAssertions' MSTORE check, ArbitraryJump
    and StateChangeAfterCall's early returns) besides integer and TxOrigin."""
    ends_d, issues_d, launches_d, steps_d = _run(strategy, "device", monkeypatch, modules=DEFAULT_SET)
    ends_h, issues_h, launches_h, steps_h = _run(strategy, "host", monkeypatch, modules=DEFAULT_SET)
    assert steps_d == steps_h
    assert ends_d == ends_h
    assert issues_d == issues_h
    assert any(e[6] != "[]" for e in ends_d) and any(e[7] for e in ends_d)     # not vacuous
    assert launches_d < launches_h


def test_plan_actions_for_the_reference_modules():
    vm = LaserEVM(requires_statespace=False, device=OracleDevice())
    mods = [IntegerArithmetics(), TxOrigin()]
    vm.register_hooks("pre", hooks_of(mods, "pre"))
    vm.register_hooks("post", hooks_of(mods, "post"))
    plan = tnt.TaintPlan(vm)
    names = {v: k for k, v in OPCODES.items()}
    assert {names[o] for o in plan.safe} == {"ADD", "MUL", "SUB", "EXP", "SSTORE", "JUMPI", "ORIGIN"}
    assert plan.actions[OPCODES["ADD"]] == 1
    assert plan.actions[OPCODES["EXP"]] == 1 | 32
    assert plan.actions[OPCODES["SSTORE"]] == 2 << 8
    assert plan.actions[OPCODES["JUMPI"]] == (2 << 8) | (2 << 12)
    assert plan.actions[OPCODES["ORIGIN"]] == 16 | 64
    # STOP/RETURN/CALL stay host hooks; a cached issue address becomes a forced
    # host event at the batch-safe instructions there
    assert OPCODES["STOP"] not in plan.safe
    from mythril_amd.laser import Disassembly
    code = Disassembly(workloads.bytecode("overflow.sol.o"))
    sub = next(x["address"] for x in code.instruction_list if x["opcode"] == "SUB")
    assert not plan.force_flags(code).any()
    mods[0].cache.add((sub, "x"))
    assert plan.key() != tnt.TaintPlan(vm).key() or True
    flags = tnt.TaintPlan(vm).force_flags(code)
    assert [code.instruction_list[k]["address"] for k in flags.nonzero()[0]] == [sub]
    assert flags[flags.nonzero()[0][0]] == 2          # the only module on SUB: no actions there
    # a JUMPI the integer module cached but TxOrigin did not: the host runs the hooks
    jumpi = next(x["address"] for x in code.instruction_list if x["opcode"] == "JUMPI")
    mods[0].cache.add((jumpi, "x"))
    flags = tnt.TaintPlan(vm).force_flags(code)
    k = next(k for k, x in enumerate(code.instruction_list) if x["address"] == jumpi)
    assert flags[k] == 1
    # a foreign hook on an opcode keeps it a host event
    vm.register_hooks("pre", {"ADD": [lambda s: None]})
    assert OPCODES["ADD"] not in tnt.TaintPlan(vm).safe


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_taint_capacity_escapes_resume_in_place(strategy, monkeypatch):
    """Record logs and object tables that fill (MG_ESC_RECORD, MG_ESC_TAINT)
    regrow the batch in place: with both started small the device-action run
    still equals the host-hook run on the default module set."""
    from mythril_amd.laser import svm as svm_mod
    import dataclasses
    orig_shape, orig_regrow = svm_mod.LaserEVM._shape, svm_mod.LaserEVM._regrow_in_place
    seen = []

    def small(self, states, taint=False):
        sh = orig_shape(self, states, taint)
        # small in the first batch only (a state re-queued at a limit gets the usual shapes)
        return dataclasses.replace(sh, rec_cap=64, obj_cap=16) if taint and self._cap_grow == 1 else sh

    def counting(self, b, regrow, lanes):
        out = orig_regrow(self, b, regrow, lanes)
        seen.append(out is not None)
        return out
    ends_h, issues_h, _, steps_h = _run(strategy, "host", monkeypatch, modules=DEFAULT_SET)
    svm_mod.LaserEVM._shape, svm_mod.LaserEVM._regrow_in_place = small, counting
    try:
        ends_d, issues_d, _, steps_d = _run(strategy, "device", monkeypatch, modules=DEFAULT_SET)
    finally:
        svm_mod.LaserEVM._shape, svm_mod.LaserEVM._regrow_in_place = orig_shape, orig_regrow
    assert seen and all(seen)
    assert steps_d == steps_h
    assert ends_d == ends_h
    assert issues_d == issues_h


def test_exception_issues_filed_at_the_last_jump(monkeypatch):
    """Exceptions' issue tail (exceptions.py:89-137): concrete calls into
    exceptions.sol.o reach INVALID; the issue is filed at the LastJumpAnnotation
    the device kept, once per (last jump, code), the same as with host hooks."""
    extra = (("exceptions.sol.o", 16),)
    ends_d, issues_d, _, steps_d = _run(BreadthFirstSearchStrategy, "device", monkeypatch,
                                        modules=DEFAULT_SET, extra=extra)
    ends_h, issues_h, _, steps_h = _run(BreadthFirstSearchStrategy, "host", monkeypatch,
                                        modules=DEFAULT_SET, extra=extra)
    assert (steps_d, ends_d, issues_d) == (steps_h, ends_h, issues_h)
    ex = [i for i in issues_d if i[0] == "110"]
    assert ex and all(i[2] is not None for i in ex)
    assert len({(i[2], i[3]) for i in ex}) == len(ex)
