"""Restatements of two reference detection modules -- TEST INFRASTRUCTURE ONLY.

The reference's modules cannot be imported here (z3, eth_abi absent), so the
taint tests drive LaserEVM with these restatements of their hook logic on the
repo's expression layer.  Class names match the reference's so the taint
registry (mythril_amd/laser/taint.py BATCH_SAFE) recognises them as it would
the originals; the device must produce the same annotations, state annotations
and issues as running every hook on the host.

* IntegerArithmetics: analysis/module/modules/integer.py:33-339 (annotation
  classes :33-61, hooks :75-85, handlers :140-306).  Issue reporting keeps the
  reference's control flow but, with no SMT backend here, decides satisfiability
  only for constant constraint sets (concrete lanes produce nothing else) and
  records (swc, ostate address, operator, end address) instead of an Issue.
* TxOrigin: dependence_on_origin.py:18-107.
* UserAssertions, Exceptions: user_assertions.py:30-126, exceptions.py:36-151,
  with the issue-filing tail (get_transaction_sequence stubbed over the
  constant constraint sets of concrete lanes; UnsatError drops the issue).
* DetectionModule.execute: analysis/module/base.py:72-96 (the cache check).
"""
from __future__ import annotations

from copy import copy
from math import ceil, log2
from typing import List, Set

from mythril_amd.smt.expr import (And, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, BitVec, Bool,
                                  Expression, If, Not, symbol_factory)


class _Base:
    """base.py:30-96 (the parts hooks reach)."""
    auto_cache = True

    def __init__(self):
        self.issues: List = []
        self.cache: Set = set()

    def reset_module(self):
        self.issues = []

    def update_cache(self, issues=None):
        for issue in issues or self.issues:
            self.cache.add((issue[1], issue[-1]))

    def execute(self, target):
        addr = target.get_current_instruction()["address"]
        if (addr, target.environment.code.bytecode) in self.cache and self.auto_cache:
            return []
        result = self._execute(target)
        if result:
            if self.auto_cache:
                self.update_cache(result)
            self.issues += result
        return result


def _sat(constraints) -> bool:
    """solver.get_model on a constant set (concrete lanes): True/False; raises
    for anything symbolic (no backend in this image)."""
    for c in constraints:
        v = c.value if isinstance(c, Bool) else bool(c)
        if v is None:
            raise NotImplementedError("symbolic constraint: no SMT backend in the tests")
        if not v:
            return False
    return True


# ---------------------------------------------------------------- integer.py
class OverUnderflowAnnotation:
    """integer.py:33-46."""

    def __init__(self, overflowing_state, operator: str, constraint) -> None:
        self.overflowing_state = overflowing_state
        self.operator = operator
        self.constraint = constraint

    def __deepcopy__(self, memodict={}):
        return copy(self)


class OverUnderflowStateAnnotation:
    """integer.py:49-61."""

    def __init__(self) -> None:
        self.overflowing_state_annotations = set()

    def __copy__(self):
        new = OverUnderflowStateAnnotation()
        new.overflowing_state_annotations = copy(self.overflowing_state_annotations)
        return new


class IntegerArithmetics(_Base):
    """integer.py:64-306."""
    swc_id = "101"
    pre_hooks = ["ADD", "MUL", "EXP", "SUB", "SSTORE", "JUMPI", "STOP", "RETURN", "CALL"]
    post_hooks: List[str] = []

    def __init__(self):
        super().__init__()
        self._ostates_satisfiable = set()
        self._ostates_unsatisfiable = set()

    def _execute(self, state):
        opcode = state.get_current_instruction()["opcode"]
        funcs = {
            "ADD": [self._handle_add], "SUB": [self._handle_sub], "MUL": [self._handle_mul],
            "SSTORE": [self._handle_sstore], "JUMPI": [self._handle_jumpi], "CALL": [self._handle_call],
            "RETURN": [self._handle_return, self._handle_transaction_end],
            "STOP": [self._handle_transaction_end], "EXP": [self._handle_exp],
        }
        results = []
        for func in funcs[opcode]:
            result = func(state)
            if result and len(result) > 0:
                results += result
        return results

    def _get_args(self, state):
        stack = state.mstate.stack
        return self._make_bitvec_if_not(stack, -1), self._make_bitvec_if_not(stack, -2)

    def _handle_add(self, state):
        op0, op1 = self._get_args(state)
        c = Not(BVAddNoOverflow(op0, op1, False))
        op0.annotate(OverUnderflowAnnotation(state, "addition", c))

    def _handle_mul(self, state):
        op0, op1 = self._get_args(state)
        c = Not(BVMulNoOverflow(op0, op1, False))
        op0.annotate(OverUnderflowAnnotation(state, "multiplication", c))

    def _handle_sub(self, state):
        op0, op1 = self._get_args(state)
        c = Not(BVSubNoUnderflow(op0, op1, False))
        op0.annotate(OverUnderflowAnnotation(state, "subtraction", c))

    def _handle_exp(self, state):
        op0, op1 = self._get_args(state)
        if (op1.symbolic is False and op1.value == 0) or (op0.symbolic is False and op0.value < 2):
            return
        if op0.symbolic and op1.symbolic:
            constraint = And(op1 > symbol_factory.BitVecVal(256, 256), op0 > symbol_factory.BitVecVal(1, 256))
        elif op0.symbolic:
            constraint = op0 >= symbol_factory.BitVecVal(2 ** ceil(256 / op1.value), 256)
        else:
            constraint = op1 >= symbol_factory.BitVecVal(ceil(256 / log2(op0.value)), 256)
        op0.annotate(OverUnderflowAnnotation(state, "exponentiation", constraint))

    @staticmethod
    def _make_bitvec_if_not(stack, index):
        value = stack[index]
        if isinstance(value, BitVec):
            return value
        if isinstance(value, Bool):
            return If(value, 1, 0)
        stack[index] = symbol_factory.BitVecVal(value, 256)
        return stack[index]

    @staticmethod
    def _handle_sstore(state) -> None:
        value = state.mstate.stack[-2]
        if not isinstance(value, Expression):
            return
        sa = _get_state_annotation(state)
        for a in value.annotations:
            if isinstance(a, OverUnderflowAnnotation):
                sa.overflowing_state_annotations.add(a)

    @staticmethod
    def _handle_jumpi(state):
        value = state.mstate.stack[-2]
        sa = _get_state_annotation(state)
        for a in value.annotations:
            if isinstance(a, OverUnderflowAnnotation):
                sa.overflowing_state_annotations.add(a)

    @staticmethod
    def _handle_call(state):
        value = state.mstate.stack[-3]
        sa = _get_state_annotation(state)
        for a in value.annotations:
            if isinstance(a, OverUnderflowAnnotation):
                sa.overflowing_state_annotations.add(a)

    @staticmethod
    def _handle_return(state) -> None:
        # concrete lanes hold bytes (no Expression) in memory: nothing to collect
        _get_state_annotation(state)

    def _handle_transaction_end(self, state):
        sa = _get_state_annotation(state)
        issues = []
        for annotation in sa.overflowing_state_annotations:
            ostate = annotation.overflowing_state
            if ostate in self._ostates_unsatisfiable:
                continue
            if ostate not in self._ostates_satisfiable:
                if _sat(list(ostate.world_state.constraints) + [annotation.constraint]):
                    self._ostates_satisfiable.add(ostate)
                else:
                    self._ostates_unsatisfiable.add(ostate)
                    continue
            if not _sat(list(state.world_state.constraints) + [annotation.constraint]):
                continue
            issues.append((self.swc_id, ostate.get_current_instruction()["address"], annotation.operator,
                           state.get_current_instruction()["address"], ostate.environment.code.bytecode))
        return issues


def _get_state_annotation(state) -> OverUnderflowStateAnnotation:
    """integer.py:326-339."""
    anns = list(state.get_annotations(OverUnderflowStateAnnotation))
    if not anns:
        sa = OverUnderflowStateAnnotation()
        state.annotate(sa)
        return sa
    return anns[0]


# ------------------------------------------------------- dependence_on_origin.py
class TxOriginAnnotation:
    """dependence_on_origin.py:18-22."""


class TxOrigin(_Base):
    """dependence_on_origin.py:25-107 (an issue is recorded as (swc, address))."""
    swc_id = "115"
    pre_hooks = ["JUMPI"]
    post_hooks = ["ORIGIN"]

    def _execute(self, state):
        issues = []
        if state.get_current_instruction()["opcode"] == "JUMPI":
            for annotation in state.mstate.stack[-2].annotations:
                if isinstance(annotation, TxOriginAnnotation):
                    issues.append((self.swc_id, state.get_current_instruction()["address"],
                                   state.environment.code.bytecode))
        else:
            state.mstate.stack[-1].annotate(TxOriginAnnotation())
        return issues


def hooks_of(modules, hook_type="pre"):
    """module/util.py:13-43 get_detection_module_hooks."""
    out = {}
    for m in modules:
        for op in (m.pre_hooks if hook_type == "pre" else m.post_hooks):
            out.setdefault(op.upper(), []).append(m.execute)
    return out


# ------------------------------------------------- more default modules (§8(f)1)
class PotentialIssuesAnnotation:
    """analysis/potential_issues.py:65-75 (no __copy__: copies share the list)."""

    def __init__(self):
        self.potential_issues = []


def get_potential_issues_annotation(state) -> PotentialIssuesAnnotation:
    """potential_issues.py:77-90."""
    for annotation in state.annotations:
        if isinstance(annotation, PotentialIssuesAnnotation):
            return annotation
    annotation = PotentialIssuesAnnotation()
    state.annotate(annotation)
    return annotation


class ArbitraryStorage(_Base):
    """arbitrary_write.py:22-75: every SSTORE files a potential issue whose
    constraint asks for the slot to hit an attacker-chosen location (recorded as
    (swc, address, constant-folded constraint value))."""
    swc_id = "124"
    pre_hooks = ["SSTORE"]
    post_hooks: List[str] = []

    def _execute(self, state):
        issues = self._analyze_state(state)
        get_potential_issues_annotation(state).potential_issues.extend(issues)

    def _analyze_state(self, state):
        write_slot = state.mstate.stack[-1]
        constraints = list(state.world_state.constraints) + [
            write_slot == symbol_factory.BitVecVal(324345425435, 256)]
        return [(self.swc_id, state.get_current_instruction()["address"],
                 tuple(c.value if isinstance(c, Bool) else c for c in constraints))]


class ArbitraryJump(_Base):
    """arbitrary_jump.py:45-112: only a symbolic jump target has work."""
    swc_id = "127"
    pre_hooks = ["JUMP", "JUMPI"]
    post_hooks: List[str] = []

    def _execute(self, state):
        jump_dest = state.mstate.stack[-1]
        if jump_dest.symbolic is False:
            return []
        return [(self.swc_id, state.get_current_instruction()["address"], state.environment.code.bytecode)]


class UnsatError(Exception):
    """mythril/exceptions.py UnsatError."""


class IssueAnnotation:
    """analysis/issue_annotation.py: the issue a detector filed on a state."""

    def __init__(self, conditions, issue, detector):
        self.conditions = conditions
        self.issue = issue
        self.detector = detector


def get_transaction_sequence(state, constraints):
    """analysis/solver.py get_transaction_sequence, stubbed: UnsatError when the
    (constant) constraint set is unsat, else the ids of the path's transactions
    (the concrete model the reference would minimise is not rebuilt here)."""
    try:
        sat = _sat(constraints)
    except NotImplementedError:          # symbolic: the SAT-only backend decides (or not)
        return get_transaction_sequence_sat(state, constraints)
    if not sat:
        raise UnsatError()
    return {"steps": [str(getattr(tx, "id", tx)) for tx in state.world_state.transaction_sequence]}


def _abi_string(data: bytes):
    """eth_abi.decode_single("string", data) for a well-formed head + tail."""
    off = int.from_bytes(data[:32], "big")
    n = int.from_bytes(data[off:off + 32], "big")
    if off + 32 + n > len(data):
        raise ValueError("short string")
    return data[off + 32: off + 32 + n].decode("utf8")


class UserAssertions(_Base):
    """user_assertions.py:30-126: an MSTORE of a value carrying the
    assertion-failed pattern, or a LOG1 with the AssertionFailed(string) topic,
    files an issue when the path's constraints have a model (the MSTORE hook is
    device-deferred, LOG1 reads memory: a host hook).  An issue is recorded as
    (swc, address, description tail, bytecode) and annotated on the state."""
    swc_id = "110"
    pre_hooks = ["LOG1", "MSTORE"]
    post_hooks: List[str] = []
    mstore_pattern = "0xcafecafecafecafecafecafecafecafecafecafecafecafecafecafecafe"
    assertion_failed_hash = 0xB42604CB105A16C8F6DB8A41E6B00C0C1B4826465E8BC504B3EB3E88B3E6A4A0

    def _execute(self, state):
        opcode = state.get_current_instruction()["opcode"]
        message = None
        if opcode == "MSTORE":
            value = state.mstate.stack[-2]
            if value.symbolic:
                return []
            if self.mstore_pattern not in hex(value.value)[:126]:
                return []
            message = "Failed property id {}".format(value.value & 0xFFFF)
        else:
            topic, size, mem_start = state.mstate.stack[-3:]
            if topic.symbolic or topic.value != self.assertion_failed_hash:
                return []
            if not mem_start.symbolic and not size.symbolic:
                try:
                    message = _abi_string(bytes(state.mstate.memory[mem_start.value + 32:
                                                                    mem_start.value + size.value]))
                except Exception:
                    pass
        try:
            seq = get_transaction_sequence(state, state.world_state.constraints)
        except UnsatError:
            return []
        tail = ("A user-provided assertion failed with the message '{}'".format(message) if message
                else "A user-provided assertion failed.")
        issue = (self.swc_id, state.get_current_instruction()["address"], tail, state.environment.code.bytecode)
        state.annotate(IssueAnnotation(conditions=[And(*state.world_state.constraints)], issue=(issue, seq),
                                       detector=self))
        return [issue]


class LastJumpAnnotation:
    """exceptions.py:21-33."""

    def __init__(self, last_jump=None):
        self.last_jump = last_jump

    def __copy__(self):
        return LastJumpAnnotation(self.last_jump)


PANIC_SIGNATURE = [78, 72, 123, 113]          # exceptions.py:20: Panic(uint256)


def is_assertion_failure(state) -> bool:
    """exceptions.py:140-151."""
    offset, length = state.mstate.stack[-1], state.mstate.stack[-2]
    if offset.symbolic or length.symbolic:
        return False
    data = state.mstate.memory[offset.value: (offset.value + length.value) & ((1 << 256) - 1)]
    return list(data[:4]) == PANIC_SIGNATURE and len(data) > 0 and data[-1] == 1


class Exceptions(_Base):
    """exceptions.py:36-137: JUMP records its address in the state's
    LastJumpAnnotation (device-deferred); INVALID and an assertion-failure
    REVERT (host hooks) file an issue at the last jump's address when the path
    has a model, unless (last jump, code) is cached (auto_cache off: the module
    caches by source location itself)."""
    swc_id = "110"
    pre_hooks = ["INVALID", "JUMP", "REVERT"]
    post_hooks: List[str] = []
    auto_cache = False

    def _execute(self, state):
        issues = self._analyze_state(state)
        for issue in issues:
            self.cache.add((issue[2], issue[-1]))          # (source_location, code)
        return issues

    def _analyze_state(self, state):
        opcode = state.get_current_instruction()["opcode"]
        address = state.get_current_instruction()["address"]
        annotations = [a for a in state.get_annotations(LastJumpAnnotation)]
        if len(annotations) == 0:
            state.annotate(LastJumpAnnotation())
            annotations = [a for a in state.get_annotations(LastJumpAnnotation)]
        if opcode == "JUMP":
            annotations[0].last_jump = address
            return []
        if opcode == "REVERT" and not is_assertion_failure(state):
            return []
        cache_address = annotations[0].last_jump
        if (cache_address, state.environment.code.bytecode) in self.cache:
            return []
        try:
            seq = get_transaction_sequence(state, state.world_state.constraints)
        except UnsatError:
            return []
        issue = (self.swc_id, address, cache_address, state.environment.code.bytecode)
        state.annotate(IssueAnnotation(conditions=[And(*state.world_state.constraints)], issue=(issue, seq),
                                       detector=self))
        return [issue]


class StateChangeCallsAnnotation:
    """state_change_external_calls.py:27-40 (made by the CALL hooks)."""


class StateChangeAfterCall(_Base):
    """state_change_external_calls.py:104-185, the SLOAD/SSTORE half: with no
    StateChangeCallsAnnotation on the state (no external call yet) they return
    at once; with one, the host runs them (recorded as an issue per access)."""
    swc_id = "107"
    pre_hooks = ["SLOAD", "SSTORE"]
    post_hooks: List[str] = []

    def _execute(self, state):
        annotations = list(state.get_annotations(StateChangeCallsAnnotation))
        if len(annotations) == 0:
            return []
        return [(self.swc_id, state.get_current_instruction()["address"], state.environment.code.bytecode)]


# ------------------------------------------------ issue confirmation (SAT only)
class ConfirmationUnknown(UnsatError):
    """A confirmation the SAT-only backend could not decide: neither a model
    nor a proof of unsat.  Modules treat it as the reference treats UnsatError
    (no issue); CONFIRMATIONS counts it apart."""


CONFIRMATIONS = {"sat": 0, "unknown": 0}


def _sat_or_unknown(call):
    """Run a get_model-style call under the SAT-only backend: a model, or
    ConfirmationUnknown (SolverBackendMissing: no candidate satisfied and no
    solver can say more)."""
    from mythril_amd.smt.solver import SolverBackendMissing
    from mythril_amd.smt.solver import UnsatError as SmtUnsat
    try:
        model = call()
    except SolverBackendMissing:
        CONFIRMATIONS["unknown"] += 1
        raise ConfirmationUnknown()
    except SmtUnsat:
        raise UnsatError()
    CONFIRMATIONS["sat"] += 1
    return model


def get_model(constraints):
    """analysis/solver.py's ``get_model`` (support/model.py:21-82) as the
    modules call it, through the product's kernel-2 path."""
    from mythril_amd.smt import solver
    return _sat_or_unknown(lambda: solver.get_model(tuple(constraints)))


def _minimisation_constraints(state, constraints):
    """analysis/solver.py:219-259 _set_minimisation_constraints: calldata size
    bound, caller / account starting-balance bounds; the minimised terms."""
    from mythril_amd.smt.expr import UGE
    ws = state.world_state
    out, minimize = list(constraints), []
    for tx in ws.transaction_sequence:
        out.append(UGE(symbol_factory.BitVecVal(5000, 256), tx.call_data.calldatasize))
        minimize.append(tx.call_data.calldatasize)
        minimize.append(tx.call_value)
        out.append(UGE(symbol_factory.BitVecVal(10 ** 21, 256), ws.starting_balances[
            tx.caller if hasattr(tx.caller, "raw") else symbol_factory.BitVecVal(int(tx.caller), 256)]))
    for account in ws.accounts.values():
        out.append(UGE(symbol_factory.BitVecVal(10 ** 20, 256), ws.starting_balances[account.address]))
    return out, tuple(minimize)


def get_transaction_sequence_sat(state, constraints):
    """analysis/solver.py:54-104 get_transaction_sequence over the SAT-only
    backend: the same tx constraints and minimised terms, through get_model
    (the backend minimises by descent, it does not prove optimality).  Returns
    {"steps": [{"input", "value", "origin", "address"}]} as
    _get_concrete_transaction builds it (solver.py:191-219)."""
    from mythril_amd.laser.transaction import ContractCreationTransaction
    from mythril_amd.smt import solver
    from mythril_amd.smt.solver import Constraints
    cons, minimize = _minimisation_constraints(state, constraints)
    model = _sat_or_unknown(lambda: solver.get_model(Constraints(cons), minimize=minimize))
    steps = []
    def word(x):
        return x if hasattr(x, "raw") else symbol_factory.BitVecVal(int(x), 256)
    for tx in state.world_state.transaction_sequence:
        cd = tx.call_data
        size = model.eval(cd.calldatasize.raw, model_completion=True).param
        data = bytes(model.eval(cd[k].raw, model_completion=True).param for k in range(min(size, 5000)))
        inp = (tx.code.raw.hex() if isinstance(tx, ContractCreationTransaction) else "") + data.hex()
        steps.append({"input": "0x" + inp,
                      "value": hex(model.eval(word(tx.call_value).raw, model_completion=True).param),
                      "origin": "0x%040x" % model.eval(word(tx.caller).raw, model_completion=True).param,
                      "address": "" if isinstance(tx, ContractCreationTransaction)
                      else hex(tx.callee_account.address.value)})
    return {"steps": steps}


# ---------------------------------------------------------------- suicide.py
class AccidentallyKillable(_Base):
    """analysis/module/modules/suicide.py:25-120: a SELFDESTRUCT any sender
    reaches is an issue; the first confirmation asks the beneficiary to be the
    attacker, the fallback drops that.  An issue is (swc, address, withdraws,
    bytecode) with the transaction sequence kept on the annotation."""
    swc_id = "106"
    pre_hooks = ["SELFDESTRUCT"]
    post_hooks: List[str] = []

    def _execute(self, state):
        from mythril_amd.laser.transaction import ACTORS, ContractCreationTransaction
        instruction = state.get_current_instruction()
        to = state.mstate.stack[-1]
        attacker = symbol_factory.BitVecVal(ACTORS["ATTACKER"], 256)
        attacker_constraints = []
        for tx in state.world_state.transaction_sequence:
            if not isinstance(tx, ContractCreationTransaction):
                attacker_constraints.append(And(tx.caller == attacker, tx.caller == tx.origin))
        try:
            try:
                constraints = list(state.world_state.constraints) + [to == attacker] + attacker_constraints
                seq = get_transaction_sequence_sat(state, constraints)
                withdraws = True
            except UnsatError:
                constraints = list(state.world_state.constraints) + attacker_constraints
                seq = get_transaction_sequence_sat(state, constraints)
                withdraws = False
        except UnsatError:
            return []
        issue = (self.swc_id, instruction["address"], withdraws, state.environment.code.bytecode)
        state.annotate(IssueAnnotation(conditions=[And(*constraints)], issue=(issue, seq), detector=self))
        return [issue]


# ------------------------------------------------ ether_thief.py + potential_issues.py
class PotentialIssue:
    """analysis/potential_issues.py:10-62 (the fields check_potential_issues uses)."""

    def __init__(self, address, swc_id, bytecode, detector, constraints=None):
        self.address = address
        self.swc_id = swc_id
        self.bytecode = bytecode
        self.detector = detector
        self.constraints = constraints or []


def check_potential_issues(state) -> None:
    """analysis/potential_issues.py:93-140: at a kept transaction end, each
    potential issue whose constraints (with the path's) have a transaction
    sequence becomes an issue of its detector; the others stay potential."""
    annotation = get_potential_issues_annotation(state)
    unsat = []
    for p in annotation.potential_issues:
        if not isinstance(p, PotentialIssue):
            unsat.append(p)
            continue
        try:
            seq = get_transaction_sequence_sat(state, list(state.world_state.constraints) + p.constraints)
        except UnsatError:
            unsat.append(p)
            continue
        issue = (p.swc_id, p.address, p.bytecode)
        state.annotate(IssueAnnotation(detector=p.detector, issue=(issue, seq),
                                       conditions=[And(*(list(state.world_state.constraints) + p.constraints))]))
        p.detector.issues.append(issue)
        p.detector.update_cache([issue])
        p.detector.sequences.append(seq)
    annotation.potential_issues = unsat


class EtherThief(_Base):
    """analysis/module/modules/ether_thief.py:23-99: after a CALL / STATICCALL,
    a potential issue when the attacker's balance can end above its starting
    balance (pre-solved with get_model); confirmed at the transaction end."""
    swc_id = "105"
    pre_hooks: List[str] = []
    post_hooks = ["CALL", "STATICCALL"]

    def __init__(self):
        super().__init__()
        self.sequences = []

    def update_cache(self, issues=None):
        for issue in issues or self.issues:
            self.cache.add((issue[1], issue[-1]))

    def _execute(self, state):
        potential = self._analyze_state(state)
        get_potential_issues_annotation(state).potential_issues.extend(potential)

    def _analyze_state(self, state):
        from mythril_amd.laser.transaction import ACTORS
        from mythril_amd.smt.expr import UGT
        state = copy(state)
        instruction = state.get_current_instruction()
        attacker = symbol_factory.BitVecVal(ACTORS["ATTACKER"], 256)
        ws = state.world_state
        constraints = list(ws.constraints) + [
            UGT(ws.balances[attacker], ws.starting_balances[attacker]),
            state.environment.sender == attacker,
            state.current_transaction.caller == state.current_transaction.origin,
        ]
        try:
            get_model(list(constraints))
        except UnsatError:
            return []
        return [PotentialIssue(address=instruction["address"] - 1, swc_id=self.swc_id,
                               bytecode=state.environment.code.bytecode, detector=self,
                               constraints=constraints)]
