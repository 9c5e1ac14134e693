"""Restatements of the reference's detection modules -- TEST INFRASTRUCTURE ONLY.

The reference's modules cannot be imported here (z3, eth_abi absent), so the
tests drive LaserEVM with these restatements of their hook logic on the repo's
expression layer.  Class names match the reference's so the taint registry
(mythril_amd/laser/taint.py BATCH_SAFE) recognises them as it would the
originals.  All fourteen modules of analysis/module/loader.py:90-110 are here,
in its registration order (``MODULE_ORDER``); each files
``Issue``/``PotentialIssue`` objects with the reference's fields (contract,
function, address, SWC id, title, bytecode, transaction sequence):

* base.py:30-96 DetectionModule.execute (the (address, code) issue cache);
* report.py:23-120 Issue, potential_issues.py:10-140 PotentialIssue and
  check_potential_issues, report.py:273-285 the report's de-duplication
  (``report_issues``);
* arbitrary_jump.py, arbitrary_write.py, delegatecall.py,
  dependence_on_predictable_vars.py, dependence_on_origin.py, ether_thief.py,
  exceptions.py, external_calls.py, integer.py, multiple_sends.py,
  state_change_external_calls.py, suicide.py, unchecked_retval.py,
  user_assertions.py (cited per class);
* the MutationPruner plugin (laser/plugin/plugins/mutation_pruner.py:28-89).

Satisfiability goes through the product's kernel-2 path
(mythril_amd.smt.solver.get_model with the SAT-only backend of tests/analyze.py):
a model, or "unknown" (SolverBackendMissing), which the modules treat as the
reference treats UnsatError -- no issue -- and which ``CONFIRMATIONS`` counts
apart.  Constraint sets of concrete paths (all constants) are decided directly.
"""
from __future__ import annotations

import traceback
from copy import copy
from math import ceil, log2
from typing import Dict, List, Optional, Set

from mythril_amd.smt.expr import (UGT, ULT, And, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, BitVec,
                                  Bool, Expression, Extract, If, Not, Or, symbol_factory)

# analysis/swc_data.py
INTEGER_OVERFLOW_AND_UNDERFLOW = "101"
UNCHECKED_RET_VAL = "104"
UNPROTECTED_ETHER_WITHDRAWAL = "105"
UNPROTECTED_SELFDESTRUCT = "106"
REENTRANCY = "107"
ASSERT_VIOLATION = "110"
DELEGATECALL_TO_UNTRUSTED_CONTRACT = "112"
MULTIPLE_SENDS = "113"
TX_ORIGIN_USAGE = "115"
TIMESTAMP_DEPENDENCE = "116"
WEAK_RANDOMNESS = "120"
WRITE_TO_ARBITRARY_STORAGE = "124"
ARBITRARY_JUMP = "127"


# ------------------------------------------------------------------ issues
class Issue:
    """report.py:23-120: the fields reports, caches and tests read."""

    def __init__(self, contract, function_name, address, swc_id, title, bytecode, severity=None,
                 description_head="", description_tail="", transaction_sequence=None, gas_used=(None, None),
                 source_location=None):
        self.contract = contract
        self.function = function_name
        self.address = address
        self.swc_id = swc_id
        self.title = title
        self.bytecode = bytecode
        self.severity = severity
        self.description_head = description_head
        self.description_tail = description_tail
        self.transaction_sequence = transaction_sequence
        self.min_gas_used, self.max_gas_used = gas_used
        self.source_location = source_location

    def key(self):
        """What distinguishes two issues of a report: SWC, address, function,
        title (report.py:273-285 keys on contract + function + address + title)."""
        return (self.swc_id, self.address, self.function, self.title)

    def __repr__(self):
        return f"Issue(swc={self.swc_id}, address={self.address}, function={self.function!r}, title={self.title!r})"


def report_issues(modules) -> List[Issue]:
    """security.retrieve_callback_issues (security.py:14-25, module order) then
    Report.append_issue (report.py:273-285): one issue per (contract, function,
    address, title), the last one appended winning its slot."""
    out: Dict[tuple, Issue] = {}
    for m in modules:
        for issue in m.issues:
            out[(issue.contract, issue.function, issue.address, issue.title)] = issue
    return list(out.values())


class PotentialIssue:
    """potential_issues.py:10-62."""

    def __init__(self, contract, function_name, address, swc_id, title, bytecode, detector, severity=None,
                 description_head="", description_tail="", constraints=None):
        self.title = title
        self.contract = contract
        self.function_name = function_name
        self.address = address
        self.description_head = description_head
        self.description_tail = description_tail
        self.severity = severity
        self.swc_id = swc_id
        self.bytecode = bytecode
        self.constraints = constraints or []
        self.detector = detector

    def _key(self):
        return (self.swc_id, self.address, self.function_name, self.title,
                tuple(c.raw if isinstance(c, Expression) else c for c in self.constraints))

    def __eq__(self, other):
        return isinstance(other, PotentialIssue) and self._key() == other._key()

    def __hash__(self):
        return hash(self._key())

    def __repr__(self):
        return f"PotentialIssue({self.swc_id}, {self.address}, {self.function_name!r})"


class PotentialIssuesAnnotation:
    """potential_issues.py:65-75 (no __copy__: copies share the list)."""

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


class IssueAnnotation:
    """analysis/issue_annotation.py: the issue a detector filed on a state."""

    def __init__(self, conditions, issue, detector):
        self.conditions = conditions
        self.issue = issue
        self.detector = detector


def check_potential_issues(state) -> None:
    """potential_issues.py:93-140: at a kept transaction end, each potential
    issue whose constraints (with the path's) have a transaction sequence
    becomes an issue of its detector; the others stay potential."""
    annotation = get_potential_issues_annotation(state)
    unsat = []
    for p in annotation.potential_issues:
        try:
            seq = get_transaction_sequence(state, list(state.world_state.constraints) + list(p.constraints))
        except UnsatError:
            unsat.append(p)
            continue
        issue = Issue(contract=p.contract, function_name=p.function_name, address=p.address, title=p.title,
                      bytecode=p.bytecode, swc_id=p.swc_id, severity=p.severity,
                      gas_used=(state.mstate.min_gas_used, state.mstate.max_gas_used),
                      description_head=p.description_head, description_tail=p.description_tail,
                      transaction_sequence=seq)
        state.annotate(IssueAnnotation(detector=p.detector, issue=issue,
                                       conditions=[And(*(list(state.world_state.constraints) + list(p.constraints)))]))
        p.detector.issues.append(issue)
        p.detector.update_cache([issue])
    annotation.potential_issues = unsat


# ------------------------------------------------------------------ base
class _Base:
    """base.py:30-96 (the parts hooks reach)."""
    auto_cache = True
    swc_id = ""
    pre_hooks: List[str] = []
    post_hooks: List[str] = []

    def __init__(self):
        self.issues: List[Issue] = []
        self.cache: Set = set()

    def reset_module(self):
        self.issues = []

    def update_cache(self, issues=None):
        for issue in issues or self.issues:
            self.cache.add((issue.address, issue.bytecode))       # (address, code hash)

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


def hooks_of(modules, hook_type="pre"):
    """module/util.py:13-43 get_detection_module_hooks."""
    out = {}
    for m in modules:
        for op in (m.pre_hooks if hook_type == "pre" else m.post_hooks):
            out.setdefault(op.upper(), []).append(m.execute)
    return out


def is_prehook() -> bool:
    """module_helpers.py:1-14 reads the caller's frame text for "pre_hook" /
    "post_hook"; here the nearest frame of LaserEVM's hook runners decides."""
    for frame in reversed(traceback.extract_stack()[:-1]):
        if "post_hook" in frame.name:
            return False
        if "pre_hook" in frame.name:
            return True
    raise AssertionError("not called from a hook")


# ------------------------------------------------------------------ solving
class UnsatError(Exception):
    """mythril/exceptions.py UnsatError."""


class ConfirmationUnknown(UnsatError):
    """A query the SAT-only backend could not decide: neither a model nor a
    proof of unsat.  Modules treat it as the reference treats UnsatError (no
    issue); CONFIRMATIONS counts it apart."""


CONFIRMATIONS = {"sat": 0, "unknown": 0, "timeout": 0, "unsat": 0}


def _constant_verdict(constraints) -> Optional[bool]:
    """True / False for a set of constants (a concrete path's), else None."""
    for c in constraints:
        v = c.value if isinstance(c, Bool) else (c if isinstance(c, bool) else None)
        if v is None:
            return None
        if not v:
            return False
    return True


def _sat_or_unknown(call):
    """Run a get_model-style call under the SAT-only backend: a model, or
    ConfirmationUnknown (SolverBackendMissing: no candidate satisfied and no
    solver can say more)."""
    from mythril_amd.smt.solver import SolverBackendMissing, SolverTimeOutException
    from mythril_amd.smt.solver import UnsatError as SmtUnsat
    try:
        model = call()
    except SolverBackendMissing:
        CONFIRMATIONS["unknown"] += 1
        raise ConfirmationUnknown()
    except SolverTimeOutException:
        # the reference's timeout is an UnsatError (exceptions.py:23): no issue
        CONFIRMATIONS["timeout"] += 1
        raise UnsatError()
    except SmtUnsat:
        CONFIRMATIONS["unsat"] += 1
        raise UnsatError()
    CONFIRMATIONS["sat"] += 1
    return model


def get_model(constraints):
    """analysis/solver.py's ``get_model`` (support/model.py:21-82) as the
    modules call it, through the product's kernel-2 path."""
    from mythril_amd.smt import solver
    constraints = list(constraints)
    v = _constant_verdict(constraints)
    if v is False:
        raise UnsatError()
    if v is True:
        return solver.Model([solver.ModelRef()])
    return _sat_or_unknown(lambda: solver.get_model(tuple(constraints)))


def _calldatasize(cd):
    """calldata.calldatasize; a concrete transaction's calldata is its bytes here
    (the reference wraps them in ConcreteCalldata)."""
    if isinstance(cd, (bytes, bytearray)):
        return symbol_factory.BitVecVal(len(cd), 256)
    return cd.calldatasize


def _minimisation_constraints(state, constraints):
    """analysis/solver.py:219-259 _set_minimisation_constraints: calldata size
    bound, caller / account starting-balance bounds; the minimised terms."""
    from mythril_amd.smt.expr import UGE
    ws = state.world_state
    out, minimize = list(constraints), []
    for tx in ws.transaction_sequence:
        size = _calldatasize(tx.call_data)
        out.append(UGE(symbol_factory.BitVecVal(5000, 256), size))
        minimize.append(size)
        minimize.append(_word(tx.call_value))
        out.append(UGE(symbol_factory.BitVecVal(10 ** 21, 256), ws.starting_balances[
            tx.caller if hasattr(tx.caller, "raw") else symbol_factory.BitVecVal(int(tx.caller), 256)]))
    for account in ws.accounts.values():
        out.append(UGE(symbol_factory.BitVecVal(10 ** 20, 256), ws.starting_balances[account.address]))
    return out, tuple(minimize)


def get_transaction_sequence(state, constraints):
    """analysis/solver.py:54-104 get_transaction_sequence: the same tx
    constraints and minimised terms, through get_model (the SAT-only backend
    minimises by descent, it does not prove optimality).  Returns
    {"steps": [{"input", "value", "origin", "address"}]} as
    _get_concrete_transaction builds it (solver.py:191-219).  A concrete
    path's constant set is decided directly (UnsatError when false) and keeps
    its transactions' ids only."""
    v = _constant_verdict(constraints)
    if v is False:
        raise UnsatError()
    if v is True and all(getattr(_calldatasize(tx.call_data), "value", None) is not None
                         for tx in state.world_state.transaction_sequence if tx.call_data is not None):
        return {"steps": [str(getattr(tx, "id", tx)) for tx in state.world_state.transaction_sequence]}
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
        if isinstance(cd, (bytes, bytearray)) or cd is None:
            data = bytes(cd or b"")
        else:
            size = model.eval(cd.calldatasize.raw, model_completion=True).param
            data = bytes(model.eval(cd[k].raw, model_completion=True).param for k in range(min(size, 5000)))
        inp = (tx.code.raw.hex() if isinstance(tx, ContractCreationTransaction) else "") + data.hex()
        steps.append({"input": "0x" + inp,
                      "value": hex(model.eval(word(tx.call_value).raw, model_completion=True).param),
                      "origin": "0x%040x" % model.eval(word(tx.caller).raw, model_completion=True).param,
                      "address": "" if isinstance(tx, ContractCreationTransaction)
                      else hex(tx.callee_account.address.value)})
    return {"steps": steps}


get_transaction_sequence_sat = get_transaction_sequence


def _attacker():
    from mythril_amd.laser.transaction import ACTORS
    return symbol_factory.BitVecVal(ACTORS["ATTACKER"], 256)


def _word(x):
    return x if isinstance(x, BitVec) else (If(x, 1, 0) if isinstance(x, Bool) else
                                            symbol_factory.BitVecVal(int(x), 256))


def _env_issue(state, swc_id, title, severity, head, tail, seq, address=None, **kw):
    return Issue(contract=state.environment.active_account.contract_name,
                 function_name=state.environment.active_function_name,
                 address=state.get_current_instruction()["address"] if address is None else address,
                 swc_id=swc_id, title=title, severity=severity, bytecode=state.environment.code.bytecode,
                 description_head=head, description_tail=tail, transaction_sequence=seq,
                 gas_used=(state.mstate.min_gas_used, state.mstate.max_gas_used), **kw)


# ------------------------------------------------------------ arbitrary_jump.py
def is_unique_jumpdest(jump_dest, state) -> bool:
    """arbitrary_jump.py:21-40."""
    try:
        model = get_model(state.world_state.constraints)
    except UnsatError:
        return True
    concrete = model.eval(jump_dest.raw, model_completion=True).param
    try:
        get_model(list(state.world_state.constraints) + [symbol_factory.BitVecVal(concrete, 256) != jump_dest])
    except UnsatError:
        return True
    return False


class ArbitraryJump(_Base):
    """arbitrary_jump.py:43-112: a symbolic jump target with more than one
    feasible value."""
    swc_id = ARBITRARY_JUMP
    pre_hooks = ["JUMP", "JUMPI"]
    post_hooks: List[str] = []

    def _execute(self, state):
        jump_dest = state.mstate.stack[-1]
        if jump_dest.symbolic is False:
            return []
        if is_unique_jumpdest(jump_dest, state) is True:
            return []
        try:
            seq = get_transaction_sequence(state, state.world_state.constraints)
        except UnsatError:
            return []
        issue = _env_issue(state, ARBITRARY_JUMP, "Jump to an arbitrary instruction", "High",
                           "The caller can redirect execution to arbitrary bytecode locations.", "", seq)
        state.annotate(IssueAnnotation(conditions=[And(*state.world_state.constraints)], issue=issue,
                                       detector=self))
        return [issue]


# ------------------------------------------------------------ arbitrary_write.py
class ArbitraryStorage(_Base):
    """arbitrary_write.py:22-75: every SSTORE files a potential issue asking
    the slot to hit an attacker-chosen location."""
    swc_id = WRITE_TO_ARBITRARY_STORAGE
    pre_hooks = ["SSTORE"]
    post_hooks: List[str] = []

    def _execute(self, state):
        get_potential_issues_annotation(state).potential_issues.extend(self._analyze_state(state))

    def _analyze_state(self, state):
        write_slot = state.mstate.stack[-1]
        constraints = list(state.world_state.constraints) + [
            write_slot == symbol_factory.BitVecVal(324345425435, 256)]
        return [PotentialIssue(contract=state.environment.active_account.contract_name,
                               function_name=state.environment.active_function_name,
                               address=state.get_current_instruction()["address"],
                               swc_id=WRITE_TO_ARBITRARY_STORAGE, title="Write to an arbitrary storage location",
                               severity="High", bytecode=state.environment.code.bytecode, detector=self,
                               description_head="The caller can write to arbitrary storage locations.",
                               constraints=constraints)]


# ------------------------------------------------------------ delegatecall.py
class ArbitraryDelegateCall(_Base):
    """delegatecall.py:22-96."""
    swc_id = DELEGATECALL_TO_UNTRUSTED_CONTRACT
    pre_hooks = ["DELEGATECALL"]
    post_hooks: List[str] = []

    def _execute(self, state):
        get_potential_issues_annotation(state).potential_issues.extend(self._analyze_state(state))

    def _analyze_state(self, state):
        from mythril_amd.laser.transaction import ContractCreationTransaction
        gas, to = state.mstate.stack[-1], state.mstate.stack[-2]
        address = state.get_current_instruction()["address"]
        constraints = [to == _attacker(), UGT(gas, symbol_factory.BitVecVal(2300, 256)),
                       state.new_bitvec("retval_{}".format(address), 256) == 1]
        for tx in state.world_state.transaction_sequence:
            if not isinstance(tx, ContractCreationTransaction):
                constraints.append(tx.caller == _attacker())
        return [PotentialIssue(contract=state.environment.active_account.contract_name,
                               function_name=state.environment.active_function_name, address=address,
                               swc_id=DELEGATECALL_TO_UNTRUSTED_CONTRACT,
                               bytecode=state.environment.code.bytecode,
                               title="Delegatecall to user-supplied address", severity="High", detector=self,
                               description_head="The contract delegates execution to another contract with a "
                                                "user-supplied address.", constraints=constraints)]


# ------------------------------------------------- dependence_on_predictable_vars.py
PREDICTABLE_OPS = ["COINBASE", "GASLIMIT", "TIMESTAMP", "NUMBER"]


class PredictableValueAnnotation:
    """dependence_on_predictable_vars.py:22-27."""

    def __init__(self, operation: str) -> None:
        self.operation = operation


class OldBlockNumberUsedAnnotation:
    """dependence_on_predictable_vars.py:30-35."""


class PredictableVariables(_Base):
    """dependence_on_predictable_vars.py:38-192: JUMPI on a predictable
    environment word; BLOCKHASH of an old block number."""
    swc_id = "{} {}".format(TIMESTAMP_DEPENDENCE, WEAK_RANDOMNESS)
    pre_hooks = ["JUMPI", "BLOCKHASH"]
    post_hooks = ["BLOCKHASH"] + PREDICTABLE_OPS

    def _execute(self, state):
        issues = []
        if is_prehook():
            opcode = state.get_current_instruction()["opcode"]
            if opcode == "JUMPI":
                for annotation in state.mstate.stack[-2].annotations:
                    if not isinstance(annotation, PredictableValueAnnotation):
                        continue
                    constraints = state.world_state.constraints
                    try:
                        seq = get_transaction_sequence(state, constraints)
                    except UnsatError:
                        continue
                    swc_id = TIMESTAMP_DEPENDENCE if "timestamp" in annotation.operation else WEAK_RANDOMNESS
                    issue = _env_issue(state, swc_id, "Dependence on predictable environment variable", "Low",
                                       "A control flow decision is made based on {}.".format(annotation.operation),
                                       annotation.operation + " is used to determine a control flow decision. ",
                                       seq)
                    state.annotate(IssueAnnotation(conditions=[And(*constraints)], issue=issue, detector=self))
                    issues.append(issue)
            elif opcode == "BLOCKHASH":
                param = state.mstate.stack[-1]
                constraint = [ULT(param, state.environment.block_number),
                              ULT(state.environment.block_number, symbol_factory.BitVecVal(2 ** 255, 256))]
                try:
                    get_model(list(state.world_state.constraints) + constraint)
                    state.annotate(OldBlockNumberUsedAnnotation())
                except UnsatError:
                    pass
        else:
            opcode = state.environment.code.instruction_list[state.mstate.pc - 1]["opcode"]
            if opcode == "BLOCKHASH":
                if list(state.get_annotations(OldBlockNumberUsedAnnotation)):
                    state.mstate.stack[-1].annotate(PredictableValueAnnotation("The block hash of a previous block"))
            else:
                state.mstate.stack[-1].annotate(
                    PredictableValueAnnotation("The block.{} environment variable".format(opcode.lower())))
        return issues


# ------------------------------------------------------- dependence_on_origin.py
class TxOriginAnnotation:
    """dependence_on_origin.py:18-22."""


class TxOrigin(_Base):
    """dependence_on_origin.py:25-107."""
    swc_id = TX_ORIGIN_USAGE
    pre_hooks = ["JUMPI"]
    post_hooks = ["ORIGIN"]

    def _execute(self, state):
        issues = []
        if state.get_current_instruction()["opcode"] == "JUMPI":
            for annotation in state.mstate.stack[-2].annotations:
                if not isinstance(annotation, TxOriginAnnotation):
                    continue
                constraints = copy(state.world_state.constraints)
                try:
                    seq = get_transaction_sequence(state, constraints)
                except UnsatError:
                    continue
                issue = _env_issue(state, TX_ORIGIN_USAGE, "Dependence on tx.origin", "Low",
                                   "Use of tx.origin as a part of authorization control.", "", seq)
                state.annotate(IssueAnnotation(conditions=[And(*constraints)], issue=issue, detector=self))
                issues.append(issue)
        else:
            state.mstate.stack[-1].annotate(TxOriginAnnotation())
        return issues


# ------------------------------------------------------------ ether_thief.py
class EtherThief(_Base):
    """ether_thief.py:23-99: after a CALL / STATICCALL, a potential issue when
    the attacker's balance can end above its starting balance (pre-solved with
    get_model); confirmed at the transaction end."""
    swc_id = UNPROTECTED_ETHER_WITHDRAWAL
    pre_hooks: List[str] = []
    post_hooks = ["CALL", "STATICCALL"]

    def _execute(self, state):
        get_potential_issues_annotation(state).potential_issues.extend(self._analyze_state(state))

    def _analyze_state(self, state):
        state = copy(state)
        instruction = state.get_current_instruction()
        ws = state.world_state
        attacker = _attacker()
        constraints = list(ws.constraints) + [
            UGT(ws.balances[attacker], ws.starting_balances[attacker]),
            state.environment.sender == attacker,
            state.current_transaction.caller == state.current_transaction.origin,
        ]
        try:
            get_model(list(constraints))
        except UnsatError:
            return []
        return [PotentialIssue(contract=state.environment.active_account.contract_name,
                               function_name=state.environment.active_function_name,
                               address=instruction["address"] - 1,      # the post hook's previous instruction
                               swc_id=UNPROTECTED_ETHER_WITHDRAWAL, title="Unprotected Ether Withdrawal",
                               severity="High", bytecode=state.environment.code.bytecode, detector=self,
                               description_head="Any sender can withdraw Ether from the contract account.",
                               constraints=constraints)]


# ------------------------------------------------------------ exceptions.py
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
    return list(data[:4]) == PANIC_SIGNATURE and data[-1] == 1


class Exceptions(_Base):
    """exceptions.py:36-137: JUMP records its address in the state's
    LastJumpAnnotation; INVALID and an assertion-failure REVERT file an issue
    when the path has a model, unless (last jump, code) is cached (auto_cache
    off: the module caches by source location)."""
    swc_id = ASSERT_VIOLATION
    pre_hooks = ["INVALID", "JUMP", "REVERT"]
    post_hooks: List[str] = []
    auto_cache = False

    def _execute(self, state):
        issues = self._analyze_state(state)
        for issue in issues:
            self.cache.add((issue.source_location, issue.bytecode))
        return issues

    def _analyze_state(self, state):
        opcode = state.get_current_instruction()["opcode"]
        address = state.get_current_instruction()["address"]
        annotations = list(state.get_annotations(LastJumpAnnotation))
        if len(annotations) == 0:
            state.annotate(LastJumpAnnotation())
            annotations = list(state.get_annotations(LastJumpAnnotation))
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
        issue = _env_issue(state, ASSERT_VIOLATION, "Exception State", "Medium",
                           "An assertion violation was triggered.", "", seq, address=address,
                           source_location=cache_address)
        state.annotate(IssueAnnotation(conditions=[And(*state.world_state.constraints)], issue=issue,
                                       detector=self))
        return [issue]


# ------------------------------------------------------------ external_calls.py
PRECOMPILE_COUNT = 9            # laser/ethereum/natives.py PRECOMPILE_COUNT


def _is_precompile_call(state) -> bool:
    """external_calls.py:30-44 (unused by the module's hook path)."""
    to = state.mstate.stack[-2]
    constraints = list(state.world_state.constraints) + [
        Or(to < symbol_factory.BitVecVal(1, 256), to > symbol_factory.BitVecVal(PRECOMPILE_COUNT, 256))]
    try:
        get_model(constraints)
        return False
    except UnsatError:
        return True


class ExternalCalls(_Base):
    """external_calls.py:47-118: a CALL forwarding more than 2300 gas to the
    attacker is a potential issue (pre-solved with get_transaction_sequence)."""
    swc_id = REENTRANCY
    pre_hooks = ["CALL"]
    post_hooks: List[str] = []

    def _execute(self, state):
        get_potential_issues_annotation(state).potential_issues.extend(self._analyze_state(state))

    def _analyze_state(self, state):
        if state.environment.active_function_name == "constructor":
            return []
        gas, to = state.mstate.stack[-1], state.mstate.stack[-2]
        address = state.get_current_instruction()["address"]
        constraints = [UGT(gas, symbol_factory.BitVecVal(2300, 256)), to == _attacker()]
        try:
            get_transaction_sequence(state, constraints + list(state.world_state.constraints))
        except UnsatError:
            return []
        return [PotentialIssue(contract=state.environment.active_account.contract_name,
                               function_name=state.environment.active_function_name, address=address,
                               swc_id=REENTRANCY, title="External Call To User-Supplied Address",
                               bytecode=state.environment.code.bytecode, severity="Low",
                               description_head="A call to a user-supplied address is executed.",
                               constraints=constraints, detector=self)]


# ------------------------------------------------------------ integer.py
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


def _get_state_annotation(state) -> OverUnderflowStateAnnotation:
    """integer.py:326-339."""
    anns = list(state.get_annotations(OverUnderflowStateAnnotation))
    if not anns:
        sa = OverUnderflowStateAnnotation()
        state.annotate(sa)
        return sa
    return anns[0]


class IntegerArithmetics(_Base):
    """integer.py:64-306."""
    swc_id = INTEGER_OVERFLOW_AND_UNDERFLOW
    pre_hooks = ["ADD", "MUL", "EXP", "SUB", "SSTORE", "JUMPI", "STOP", "RETURN", "CALL"]
    post_hooks: List[str] = []

    def __init__(self):
        super().__init__()
        self._ostates_satisfiable = set()
        self._ostates_unsatisfiable = set()

    def reset_module(self):
        super().reset_module()
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
    def _collect(state, value):
        sa = _get_state_annotation(state)
        for a in value.annotations:
            if isinstance(a, OverUnderflowAnnotation):
                sa.overflowing_state_annotations.add(a)

    @staticmethod
    def _handle_sstore(state) -> None:
        value = state.mstate.stack[-2]
        if not isinstance(value, Expression):
            return
        IntegerArithmetics._collect(state, value)

    @staticmethod
    def _handle_jumpi(state):
        IntegerArithmetics._collect(state, state.mstate.stack[-2])

    @staticmethod
    def _handle_call(state):
        IntegerArithmetics._collect(state, state.mstate.stack[-3])

    @staticmethod
    def _handle_return(state) -> None:
        """integer.py:220-240: the annotations of the returned memory bytes."""
        offset, length = state.mstate.stack[-1], state.mstate.stack[-2]
        sa = _get_state_annotation(state)
        if offset.symbolic or length.symbolic:
            elements = state.mstate.memory[offset: offset + length]
        else:
            elements = state.mstate.memory[offset.value: offset.value + length.value]
        for element in elements:
            if not isinstance(element, Expression):
                continue
            for a in element.annotations:
                if isinstance(a, OverUnderflowAnnotation):
                    sa.overflowing_state_annotations.add(a)

    def _handle_transaction_end(self, state):
        sa = _get_state_annotation(state)
        issues = []
        for annotation in sa.overflowing_state_annotations:
            ostate = annotation.overflowing_state
            if ostate in self._ostates_unsatisfiable:
                continue
            if ostate not in self._ostates_satisfiable:
                try:
                    get_model(list(ostate.world_state.constraints) + [annotation.constraint])
                    self._ostates_satisfiable.add(ostate)
                except Exception:                   # integer.py:261: a bare except
                    self._ostates_unsatisfiable.add(ostate)
                    continue
            try:
                constraints = list(state.world_state.constraints) + [annotation.constraint]
                seq = get_transaction_sequence(state, constraints)
            except UnsatError:
                continue
            issue = Issue(contract=ostate.environment.active_account.contract_name,
                          function_name=ostate.environment.active_function_name,
                          address=ostate.get_current_instruction()["address"],
                          swc_id=INTEGER_OVERFLOW_AND_UNDERFLOW, bytecode=ostate.environment.code.bytecode,
                          title="Integer Arithmetic Bugs", severity="High",
                          description_head="The arithmetic operator can {}.".format(
                              "underflow" if annotation.operator == "subtraction" else "overflow"),
                          gas_used=(state.mstate.min_gas_used, state.mstate.max_gas_used),
                          transaction_sequence=seq)
            issue.operator = annotation.operator
            state.annotate(IssueAnnotation(issue=issue, detector=self, conditions=[And(*constraints)]))
            issues.append(issue)
        return issues


# ------------------------------------------------------------ multiple_sends.py
class MultipleSendsAnnotation:
    """multiple_sends.py:17-25."""

    def __init__(self) -> None:
        self.call_offsets: List[int] = []

    def __copy__(self):
        result = MultipleSendsAnnotation()
        result.call_offsets = copy(self.call_offsets)
        return result


class MultipleSends(_Base):
    """multiple_sends.py:28-102: every call after the first in one transaction."""
    swc_id = MULTIPLE_SENDS
    pre_hooks = ["CALL", "DELEGATECALL", "STATICCALL", "CALLCODE", "RETURN", "STOP"]
    post_hooks: List[str] = []

    def _execute(self, state):
        instruction = state.get_current_instruction()
        annotations = list(state.get_annotations(MultipleSendsAnnotation))
        if len(annotations) == 0:
            state.annotate(MultipleSendsAnnotation())
            annotations = list(state.get_annotations(MultipleSendsAnnotation))
        call_offsets = annotations[0].call_offsets
        if instruction["opcode"] in ("CALL", "DELEGATECALL", "STATICCALL", "CALLCODE"):
            call_offsets.append(instruction["address"])
            return []
        for offset in call_offsets[1:]:
            try:
                seq = get_transaction_sequence(state, state.world_state.constraints)
            except UnsatError:
                continue
            issue = _env_issue(state, MULTIPLE_SENDS, "Multiple Calls in a Single Transaction", "Low",
                               "Multiple calls are executed in the same transaction.", "", seq, address=offset)
            state.annotate(IssueAnnotation(conditions=[And(*state.world_state.constraints)], issue=issue,
                                           detector=self))
            return [issue]
        return []


# ------------------------------------------------- state_change_external_calls.py
CALL_LIST = ["CALL", "DELEGATECALL", "CALLCODE"]
STATE_READ_WRITE_LIST = ["SSTORE", "SLOAD", "CREATE", "CREATE2"]


class StateChangeCallsAnnotation:
    """state_change_external_calls.py:27-106."""

    def __init__(self, call_state, user_defined_address: bool) -> None:
        self.call_state = call_state
        self.state_change_states = []
        self.user_defined_address = user_defined_address

    def __copy__(self):
        new = StateChangeCallsAnnotation(self.call_state, self.user_defined_address)
        new.state_change_states = self.state_change_states[:]
        return new

    def get_issue(self, global_state, detector) -> Optional[PotentialIssue]:
        if not self.state_change_states:
            return None
        gas, to = self.call_state.mstate.stack[-1], self.call_state.mstate.stack[-2]
        constraints = [UGT(gas, symbol_factory.BitVecVal(2300, 256)),
                       Or(to > symbol_factory.BitVecVal(16, 256), to == symbol_factory.BitVecVal(0, 256))]
        if self.user_defined_address:
            constraints.append(to == symbol_factory.BitVecVal(0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF, 256))
        try:
            get_transaction_sequence(global_state, constraints + list(global_state.world_state.constraints))
        except UnsatError:
            return None
        read_or_write = "Read of" if global_state.get_current_instruction()["opcode"] == "SLOAD" else "Write to"
        return PotentialIssue(contract=global_state.environment.active_account.contract_name,
                              function_name=global_state.environment.active_function_name,
                              address=global_state.get_current_instruction()["address"],
                              title="State access after external call",
                              severity="Medium" if self.user_defined_address else "Low",
                              description_head="{} persistent state following external call".format(read_or_write),
                              swc_id=REENTRANCY, bytecode=global_state.environment.code.bytecode,
                              constraints=constraints, detector=detector)


class StateChangeAfterCall(_Base):
    """state_change_external_calls.py:109-205."""
    swc_id = REENTRANCY
    pre_hooks = CALL_LIST + STATE_READ_WRITE_LIST
    post_hooks: List[str] = []

    def _execute(self, state):
        get_potential_issues_annotation(state).potential_issues.extend(self._analyze_state(state))

    @staticmethod
    def _add_external_call(global_state) -> None:
        gas, to = global_state.mstate.stack[-1], global_state.mstate.stack[-2]
        try:
            constraints = list(global_state.world_state.constraints)
            get_model(constraints + [UGT(gas, symbol_factory.BitVecVal(2300, 256)),
                                     Or(to > symbol_factory.BitVecVal(16, 256),
                                        to == symbol_factory.BitVecVal(0, 256))])
            try:
                constraints += [to == symbol_factory.BitVecVal(0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF, 256)]
                get_model(constraints)
                global_state.annotate(StateChangeCallsAnnotation(global_state, True))
            except UnsatError:
                global_state.annotate(StateChangeCallsAnnotation(global_state, False))
        except UnsatError:
            pass

    def _analyze_state(self, global_state):
        if global_state.environment.active_function_name == "constructor":
            return []
        annotations = list(global_state.get_annotations(StateChangeCallsAnnotation))
        op_code = global_state.get_current_instruction()["opcode"]
        if len(annotations) == 0 and op_code in STATE_READ_WRITE_LIST:
            return []
        if op_code in STATE_READ_WRITE_LIST:
            for annotation in annotations:
                annotation.state_change_states.append(global_state)
        if op_code in CALL_LIST:
            value = global_state.mstate.stack[-3]
            if StateChangeAfterCall._balance_change(value, global_state):
                for annotation in annotations:
                    annotation.state_change_states.append(global_state)
            StateChangeAfterCall._add_external_call(global_state)
        out = []
        for annotation in annotations:
            if not annotation.state_change_states:
                continue
            issue = annotation.get_issue(global_state, self)
            if issue:
                out.append(issue)
        return out

    @staticmethod
    def _balance_change(value, global_state) -> bool:
        if not value.symbolic:
            return value.value > 0
        try:
            get_model(list(global_state.world_state.constraints) + [value > symbol_factory.BitVecVal(0, 256)])
            return True
        except UnsatError:
            return False


# ---------------------------------------------------------------- suicide.py
class AccidentallyKillable(_Base):
    """analysis/module/modules/suicide.py:25-120: a SELFDESTRUCT any sender
    reaches; the first confirmation asks the beneficiary to be the attacker,
    the fallback drops that."""
    swc_id = UNPROTECTED_SELFDESTRUCT
    pre_hooks = ["SELFDESTRUCT"]
    post_hooks: List[str] = []

    def _execute(self, state):
        from mythril_amd.laser.transaction import ContractCreationTransaction
        instruction = state.get_current_instruction()
        to = state.mstate.stack[-1]
        attacker = _attacker()
        attacker_constraints = []
        for tx in state.world_state.transaction_sequence:
            if not isinstance(tx, ContractCreationTransaction):
                attacker_constraints.append(And(tx.caller == attacker, tx.caller == tx.origin))
        try:
            try:
                constraints = list(state.world_state.constraints) + [to == attacker] + attacker_constraints
                seq = get_transaction_sequence(state, constraints)
                withdraws = True
            except UnsatError:
                constraints = list(state.world_state.constraints) + attacker_constraints
                seq = get_transaction_sequence(state, constraints)
                withdraws = False
        except UnsatError:
            return []
        issue = _env_issue(state, UNPROTECTED_SELFDESTRUCT, "Unprotected Selfdestruct", "High",
                           "Any sender can cause the contract to self-destruct.", "", seq,
                           address=instruction["address"])
        issue.withdraws = withdraws
        state.annotate(IssueAnnotation(conditions=[And(*constraints)], issue=issue, detector=self))
        return [issue]


# ------------------------------------------------------------ unchecked_retval.py
class UncheckedRetvalAnnotation:
    """unchecked_retval.py:28-36."""

    def __init__(self) -> None:
        self.retvals: List[dict] = []

    def __copy__(self):
        result = UncheckedRetvalAnnotation()
        result.retvals = copy(self.retvals)
        return result


class UncheckedRetval(_Base):
    """unchecked_retval.py:39-142: a call's return value that can be 0 and 1
    at the transaction's end."""
    swc_id = UNCHECKED_RET_VAL
    pre_hooks = ["STOP", "RETURN"]
    post_hooks = ["CALL", "DELEGATECALL", "STATICCALL", "CALLCODE"]

    def _execute(self, state):
        instruction = state.get_current_instruction()
        annotations = list(state.get_annotations(UncheckedRetvalAnnotation))
        if len(annotations) == 0:
            state.annotate(UncheckedRetvalAnnotation())
            annotations = list(state.get_annotations(UncheckedRetvalAnnotation))
        retvals = annotations[0].retvals
        if instruction["opcode"] in ("STOP", "RETURN"):
            issues = []
            for retval in retvals:
                try:
                    get_transaction_sequence(state, list(state.world_state.constraints) + [retval["retval"] == 1])
                    seq = get_transaction_sequence(state, list(state.world_state.constraints) +
                                                   [retval["retval"] == 0])
                except UnsatError:
                    continue
                issue = _env_issue(state, UNCHECKED_RET_VAL, "Unchecked return value from external call.", "Medium",
                                   "The return value of a message call is not checked.", "", seq,
                                   address=retval["address"])
                conditions = [And(*(list(state.world_state.constraints) + [retval["retval"] == 1])),
                              And(*(list(state.world_state.constraints) + [retval["retval"] == 0]))]
                state.annotate(IssueAnnotation(conditions=conditions, issue=issue, detector=self))
                issues.append(issue)
            return issues
        if state.environment.code.instruction_list[state.mstate.pc - 1]["opcode"] not in (
                "CALL", "DELEGATECALL", "STATICCALL", "CALLCODE"):
            return []
        retvals.append({"address": state.instruction["address"] - 1, "retval": state.mstate.stack[-1]})
        return []


# ------------------------------------------------------------ user_assertions.py
def _abi_string(data: bytes):
    """eth_abi.decode_single("string", data) for a well-formed head + tail."""
    off = int.from_bytes(data[:32], "big")
    n = int.from_bytes(data[off:off + 32], "big")
    if off + 32 + n > len(data):
        raise ValueError("short string")
    return data[off + 32: off + 32 + n].decode("utf8")


class UserAssertions(_Base):
    """user_assertions.py:30-126: an MSTORE of a value carrying the
    assertion-failed pattern, or a LOG1 with the AssertionFailed(string)
    topic, files an issue when the path's constraints have a model."""
    swc_id = ASSERT_VIOLATION
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
        issue = _env_issue(state, ASSERT_VIOLATION, "Exception State", "Medium",
                           "A user-provided assertion failed.", tail, seq)
        state.annotate(IssueAnnotation(conditions=[And(*state.world_state.constraints)], issue=issue,
                                       detector=self))
        return [issue]


# ------------------------------------------------------------ loader.py
MODULE_ORDER = ["ArbitraryJump", "ArbitraryStorage", "ArbitraryDelegateCall", "PredictableVariables", "TxOrigin",
                "EtherThief", "Exceptions", "ExternalCalls", "IntegerArithmetics", "MultipleSends",
                "StateChangeAfterCall", "AccidentallyKillable", "UncheckedRetval", "UserAssertions"]


def detection_modules(white_list=None):
    """ModuleLoader().get_detection_modules(EntryPoint.CALLBACK, white_list)
    (loader.py:50-88): fresh instances in registration order."""
    names = MODULE_ORDER if not white_list else [n for n in MODULE_ORDER if n in white_list]
    return [globals()[n]() for n in names]


# ------------------------------------------------------------ plugins
class MutationAnnotation:
    """plugin_annotations.py:13-25."""
    persist_over_calls = True


class MutationPruner:
    """laser/plugin/plugins/mutation_pruner.py:28-89: a message call that
    executed no SSTORE / CALL / STATICCALL and cannot have received value adds
    no world state."""

    def initialize(self, laser) -> None:
        from mythril_amd.laser.signals import PluginSkipWorldState
        from mythril_amd.laser.transaction import ContractCreationTransaction

        def mutator(state):
            state.annotate(MutationAnnotation())
        for op in ("SSTORE", "CALL", "STATICCALL"):
            laser.pre_hook(op)(mutator)

        def world_state_filter_hook(state):
            if isinstance(state.current_transaction, ContractCreationTransaction):
                return
            callvalue = state.environment.callvalue
            if not isinstance(callvalue, Expression):
                callvalue = symbol_factory.BitVecVal(int(callvalue), 256)
            try:
                get_model(list(state.world_state.constraints) + [UGT(callvalue, symbol_factory.BitVecVal(0, 256))])
                return
            except UnsatError:
                pass
            if len(list(state.get_annotations(MutationAnnotation))) == 0:
                raise PluginSkipWorldState
        laser.register_laser_hooks("add_world_state", world_state_filter_hook)
