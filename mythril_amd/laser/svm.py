"""LaserEVM for the MI355X batched core — the drop-in for the reference's
``LaserEVM.exec`` / ``execute_state`` loop (laser/ethereum/svm.py:293-491).

Same constructor arguments, same hook API (``register_hooks``,
``register_laser_hooks``, ``register_instr_hooks``, ``laser_hook``, ``pre_hook``,
``post_hook``, ``instr_hook``; the 11 laser hook types of svm.py:128-140), same
``exec(create, track_gas)`` contract, same ``open_states`` / ``work_list`` /
``total_states`` bookkeeping.  What differs is who steps the paths: every state
of the work list becomes one lane of kernel 1 (libmythgpu.so); the host only
sees a path when the reference would run host code for it:

* before an opcode that has an svm pre/post hook or an instruction hook
  (the lane stops with MG_HOOK; hooks fire on the materialised GlobalState;
  the lane resumes with MG_LANE_HOOK_ACK and, when post hooks exist,
  MG_LANE_STEP1 so they fire on the successor);
* when the path ends (STOP/RETURN/REVERT/past-the-end/VmException/dropped
  JUMPI): ``transaction_end`` hooks, ``_add_world_state``, ``final_states``;
* when the opcode needs semantics outside the concrete subset (MG_ESCAPE):
  the state is handed to ``escape_handler`` (in an integration, the
  reference's own ``execute_state``); without one it is dropped exactly as
  svm.py:314-316 drops a NotImplementedError.

Event order.  The reference pops one state per iteration; for concrete paths
(one successor each) BFS advances every path one instruction per round and DFS
runs the newest path to its end first.  Kernel 1 runs the paths independently,
so the host re-serialises the events: under BFS it delivers them by
(instruction round, work-list position), pausing lanes at a step horizon
(``mg_step_until``) so no path runs past an undelivered earlier event; under
DFS by (reverse position, round).  Hooks therefore fire in the reference's
order, and ``open_states`` / ``final_states`` come out in the reference's
order.  Hook-free paths run in one launch.
"""
from __future__ import annotations

import bisect
import dataclasses
import gc
import heapq
import itertools
import logging
import os
import random
import sys
from collections import Counter, defaultdict
from copy import copy
from datetime import datetime, timedelta
from typing import Callable, DefaultDict, Dict, List, Optional, Tuple

import numpy as np

from ..lanes import (LaneBatch, LaneShape, MG_DEPTH, MG_ENV_WORDS, MG_ESCAPE, MG_ESC_MEMORY,
                     MG_ESC_RECORD, MG_ESC_STACK, MG_ESC_STORAGE, MG_ESC_TRACE, MG_ESC_ARENA,
                     MG_ESC_SYMBOLIC, MG_ESC_TAINT, MG_FORK, MG_LANE_BALANCE, MG_LANE_SYMBOLIC, MG_LANE_TAINT,
                     MG_EXC_STACK_UNDERFLOW,
                     MG_HALT_DROPPED, MG_LOOP_BOUND,
                     MG_HALT_END, MG_HALT_RETURN, MG_HALT_REVERT, MG_HALT_STOP, MG_HOOK,
                     MG_LANE_CREATION, MG_LANE_HOOK_ACK, MG_LANE_RETDATA, MG_LANE_STATIC, MG_LANE_STEP1, MG_RUNNING, MG_VMEXC,
                     MG_STACK_LIMIT, MG_FENT_NONE,
                     limbs_to_word, rows_to_words, word_to_limbs)
from ..smt.exponent_manager import exponent_function_manager
from ..smt.expr import ConstWord, Expression, symbol_factory
from ..smt.keccak_manager import keccak_function_manager
from ..smt import solver as solver_mod
from ..smt.solver import Constraints, SnapshotConstraints, SolverBackendMissing, args, query_raw
from .opcodes import ADDRESS_OPCODE_MAPPING, OPCODES, get_required_stack_elements
from .signals import PluginSkipState, PluginSkipWorldState
from .state import GlobalState, LazyStack, Memory, MachineStack, concrete
from .cfg import Edge, JumpType, Node, NodeFlags
from .strategy import DelayConstraintStrategy, DepthFirstSearchStrategy, JumpdestCountAnnotation
from . import symbolic as sym
from . import taint as tnt
from .transaction import ContractCreationTransaction, install_runtime_code

log = logging.getLogger(__name__)

# opcodes _ack_safe may defer, with the number of words the real pop takes
# (ADDMOD/MULMOD 3, DUPk k, SWAPk k+1: the reference's precheck table says less)
_ACK_SAFE: Dict[str, int] = {
    **{op: 2 for op in ("ADD", "MUL", "SUB", "DIV", "SDIV", "MOD", "SMOD", "SIGNEXTEND", "LT", "GT",
                        "SLT", "SGT", "EQ", "AND", "OR", "XOR", "BYTE", "SHL", "SHR", "SAR",
                        "MSTORE", "MSTORE8", "SSTORE", "JUMPI")},
    "ADDMOD": 3, "MULMOD": 3, "ISZERO": 1, "NOT": 1, "POP": 1, "MLOAD": 1, "SLOAD": 1, "JUMP": 1,
    "JUMPDEST": 0,
    **{f"PUSH{k}": 0 for k in range(1, 33)},
    **{f"DUP{k}": k for k in range(1, 17)},
    **{f"SWAP{k}": k + 1 for k in range(1, 17)},
}

_EXEC_DEPTH = 0         # nesting of LaserEVM.exec drains (the outermost resets the lane term table)
_MERGE_GAP = 256        # lanes: transfer ranges closer than this merge into one copy
_EXECUTED_HALTS = (MG_HALT_STOP, MG_HALT_RETURN, MG_HALT_REVERT, MG_VMEXC, MG_HALT_DROPPED)
_INF = float("inf")
_NO_GAS_LIMIT = (1 << 64) - 1


class _Lane:
    __slots__ = ("state", "pos", "phase", "dirty")

    def __init__(self, state: GlobalState, pos: int):
        self.state = state
        self.pos = pos
        self.phase = "run"        # run (on device) | event | paused | done
        self.dirty = False        # host image changed, upload before the next launch


class LaserEVM:
    """The LASER engine with kernel 1 stepping every path of the work list."""

    _fast_hooks = True      # plain lanes' pre-hook events take _deliver_plain_hook
    # The reference's evaluate() steps a copy of every hooked state
    # (instructions.py:121-130).  The batched core copies only when a hook kept
    # a reference to the state or to a part the lane changes in place (_held:
    # the state, machine state, stack, memory, world state, constraint and
    # annotation lists, environment, active account, storage, transaction
    # stack, annotations).  Contract for hooks: keep what you need by
    # reference to one of those objects (or copy it); a hook that swaps one
    # kept reference for another of the same objects, or keeps an inner word
    # it later mutates in place, must run with always_copy_hooked = True.
    always_copy_hooked = False

    def __init__(self, dynamic_loader=None, max_depth=float("inf"), execution_timeout=60,
                 create_timeout=10, strategy=DepthFirstSearchStrategy, transaction_count=2,
                 requires_statespace=True, iprof=None, use_reachability_check=True,
                 beam_width=None, device=None, escape_handler: Optional[Callable] = None):
        self.execution_info: List = []
        self.open_states: List = []
        self.total_states = 0
        self.dynamic_loader = dynamic_loader
        self.use_reachability_check = use_reachability_check

        self.work_list: List[GlobalState] = []
        self.device_ms = 0.0            # kernel-1 time of every launch exec() issued
        self.strategy = strategy(self.work_list, max_depth, beam_width=beam_width)
        self.max_depth = max_depth
        self.transaction_count = transaction_count

        self.execution_timeout = execution_timeout or 0
        self.create_timeout = create_timeout or 0

        # the statespace graph (svm.py:94-97, cfg.py): with requires_statespace
        # exec() steps every state one instruction at a time (_exec_stepwise) so
        # that each node lists its states; without it the lanes run free and the
        # graph stays empty
        self.requires_statespace = requires_statespace
        self.nodes: Dict[int, Node] = {}
        self.edges: List[Edge] = []

        self.time: Optional[datetime] = None
        self.executed_transactions = False

        self.pre_hooks: DefaultDict[str, List[Callable]] = defaultdict(list)
        self.post_hooks: DefaultDict[str, List[Callable]] = defaultdict(list)

        self._add_world_state_hooks: List[Callable] = []
        self._execute_state_hooks: List[Callable] = []
        self._start_exec_trans_hooks: List[Callable] = []
        self._stop_exec_trans_hooks: List[Callable] = []
        self._start_sym_trans_hooks: List[Callable] = []
        self._stop_sym_trans_hooks: List[Callable] = []
        self._start_sym_exec_hooks: List[Callable] = []
        self._stop_sym_exec_hooks: List[Callable] = []
        self._start_exec_hooks: List[Callable] = []
        self._stop_exec_hooks: List[Callable] = []
        self._transaction_end_hooks: List[Callable] = []

        self.iprof = iprof
        self.instr_pre_hook: Dict[str, List[Callable]] = {op: [] for op in OPCODES}
        self.instr_post_hook: Dict[str, List[Callable]] = {op: [] for op in OPCODES}
        self.hook_type_map = {
            "start_execute_transactions": self._start_exec_trans_hooks,
            "stop_execute_transactions": self._stop_exec_trans_hooks,
            "add_world_state": self._add_world_state_hooks,
            "execute_state": self._execute_state_hooks,
            "start_sym_exec": self._start_sym_exec_hooks,
            "stop_sym_exec": self._stop_sym_exec_hooks,
            "start_sym_trans": self._start_sym_trans_hooks,
            "stop_sym_trans": self._stop_sym_trans_hooks,
            "start_exec": self._start_exec_hooks,
            "stop_exec": self._stop_exec_hooks,
            "transaction_end": self._transaction_end_hooks,
        }
        # batched-core specifics
        self._single_step = False           # execute_state: no manage_cfg (exec() runs it)
        self._device = device
        self.escape_handler = escape_handler
        self.record_coverage = False        # set by the coverage plugin
        self.lane_steps = 0                 # device instructions executed by exec()
        self.launches = 0
        self._exec_stop = False
        self.forks = 0                      # symbolic JUMPIs the device stopped at (MG_FORK)
        self.escapes_dropped = 0            # escaped states dropped for want of an escape handler
        self.regrows = 0                    # capacity escapes resumed in a regrown batch
        self._code_ids: Dict[bytes, int] = {}
        self._code_objs: Dict[bytes, object] = {}
        # coverage the reference's execute_state hook records for states the
        # device never executes (escaped, skipped by a pre hook)
        self._host_cov: Dict[bytes, set] = defaultdict(set)
        self._jd_addrs: Dict[str, List[int]] = {}     # jump checks of _ack_safe
        # coverage other ranks reported (sharded runs, laser/sharded.py), OR-ed in
        self._peer_cov: Dict[str, np.ndarray] = {}
        self._cap_grow = 1
        # taint lanes (laser/taint.py): force object tracking even without
        # annotating hooks (a caller that annotates words itself sets this)
        self.track_objects = False
        self._plan: Optional[tnt.TaintPlan] = None
        self._tl: Optional[List[tnt.LaneTaint]] = None
        # fork filters of consecutive MG_FORK events, evaluated together (one
        # kernel-2 launch per group) before anything else can observe them
        self._pending_forks: List = []
        # a fork-filter query no quick-sat candidate answers and no SMT backend
        # can decide: "raise" (SolverBackendMissing) or "keep" the successor
        # (prefilter-only runs, without smt.exact behind kernel 2; counted in fork_stats)
        self.unknown_forks = "raise"
        self.fork_stats = {"groups": 0, "queries": 0, "kept": 0, "pruned": 0, "unknown": 0, "flushes": 0}
        log.info("LASER EVM (MI355X batched core) initialized")

    # ------------------------------------------------------------- device
    @property
    def device(self):
        if self._device is None:
            from ..device import GpuDevice
            self._device = GpuDevice(int(os.environ.get("LOCAL_RANK", "0")))
        return self._device

    def code_id(self, code) -> int:
        raw = code.raw
        cid = self._code_ids.get(raw)
        if cid is None:
            cid = self.device.load_code(raw)
            self._code_ids[raw] = cid
            self._code_objs[raw] = code
        return cid

    # ------------------------------------------------------------- strategy / timeouts
    def extend_strategy(self, extension, **kwargs) -> None:
        self.strategy = extension(self.strategy, **kwargs)

    def _check_create_termination(self) -> bool:
        if len(self.open_states) != 0:
            return (self.create_timeout > 0 and self.time is not None
                    and self.time + timedelta(seconds=self.create_timeout) <= datetime.now())
        return self._check_execution_termination()

    def _check_execution_termination(self) -> bool:
        return (self.execution_timeout > 0 and self.time is not None
                and self.time + timedelta(seconds=self.execution_timeout) <= datetime.now())

    # ------------------------------------------------------------- exec
    def exec(self, create=False, track_gas=False) -> Optional[List[GlobalState]]:
        """svm.py:293-337: drain the work list; returns the final states when
        track_gas, else None.  Objects that exist when the drain starts are
        frozen out of the cyclic collector until it ends (gc.freeze): the event
        loop allocates a few objects per event, and every full collection it
        triggered walked the whole heap (the caller's states and everything
        else alive) again."""
        frozen = gc.get_freeze_count() == 0      # nested or caller-frozen: leave it to them
        if frozen:
            gc.freeze()
        global _EXEC_DEPTH
        if _EXEC_DEPTH == 0:
            sym.reset_terms()                    # no lane image outlives a drain
        _EXEC_DEPTH += 1
        try:
            return self._exec(create, track_gas)
        finally:
            _EXEC_DEPTH -= 1
            if frozen:
                gc.unfreeze()

    def _exec(self, create=False, track_gas=False) -> Optional[List[GlobalState]]:
        if self.requires_statespace:
            return self._exec_stepwise(create, track_gas)
        final_states: List[GlobalState] = []
        self._exec_stop = False
        for hook in self._start_exec_hooks:
            hook()
        while True:
            states = self.strategy.drain()
            if not states:
                break
            states = self._host_only(states, final_states, track_gas)
            if not states:
                continue
            leftover = self._run_batch(states, final_states, create, track_gas)
            if leftover is not None:       # timeout: the reference returns at once
                return final_states + leftover if track_gas else None
            if self._exec_stop:            # BoundedLoops popped a past-the-end state
                self._exec_stop = False
                self.work_list.clear()
                break
        for hook in self._stop_exec_hooks:
            hook()
        return final_states if track_gas else None

    def _exec_stepwise(self, create=False, track_gas=False) -> Optional[List[GlobalState]]:
        """svm.py:293-337 as written, for the statespace graph: pop one state in
        the strategy's order, step it one instruction on the device (a one-lane
        batch, execute_state's path; a state no lane can carry takes the escape
        handler), then manage_cfg on its successors.  Each node thereby holds the
        state at every instruction it covers (cfg.py Node.states)."""
        final_states: List[GlobalState] = []
        self._exec_stop = False
        for hook in self._start_exec_hooks:
            hook()
        queue: List[GlobalState] = []
        while True:
            if isinstance(self.strategy, DelayConstraintStrategy):
                if not queue:
                    queue = self.strategy.drain()
                if not queue:
                    break
                state = queue.pop(0)
            else:
                state = None
                while self.work_list:
                    cand = self.work_list.pop() if self.strategy.order == "dfs" else self.work_list.pop(0)
                    if cand.mstate.depth < self.max_depth:
                        state = cand
                        break
                if state is None:
                    break
            if create and self._check_create_termination():
                return final_states + [state] if track_gas else None
            if not create and self._check_execution_termination():
                return final_states + [state] if track_gas else None
            op = _opcode_at(state)
            saved = self.work_list[:]
            del self.work_list[:]
            self._single_step = True
            try:
                if self._host_only([state], final_states, track_gas):
                    self._run_batch([state], final_states, create, track_gas, single_step=True)
                self._flush_forks()
            finally:
                self._single_step = False
            new_states = self.work_list[:]
            self.work_list[:] = saved
            self.manage_cfg(op, new_states, parent=state)
            self.work_list.extend(new_states)
            if self._exec_stop:
                self._exec_stop = False
                self.work_list.clear()
                break
        for hook in self._stop_exec_hooks:
            hook()
        return final_states if track_gas else None

    # ------------------------------------------------------------- transactions
    def sym_exec(self, world_state=None, target_address=None, creation_code=None,
                 contract_name=None) -> None:
        """svm.py:142-212: analyse a preconfigured world state (message calls
        to ``target_address``) or, in scratch mode, run the symbolic creation
        of ``creation_code`` and then the message calls to the new account."""
        from .transaction import execute_symbolic_contract_creation
        pre_configuration_mode = target_address is not None
        scratch_mode = creation_code is not None and contract_name is not None
        if pre_configuration_mode == scratch_mode:
            raise ValueError("Symbolic execution started with invalid parameters")
        for hook in self._start_sym_exec_hooks:
            hook()
        solver_mod.time_handler.start_execution(self.execution_timeout)
        self.time = datetime.now()
        if pre_configuration_mode:
            self.open_states = [world_state]
            self.execute_transactions(symbol_factory.BitVecVal(concrete(target_address), 256))
        else:
            created = execute_symbolic_contract_creation(self, creation_code, contract_name,
                                                         world_state=world_state)
            if len(self.open_states) == 0:
                log.warning("No contract was created during the execution of contract creation")
            self.execute_transactions(created.address)
        for hook in self._stop_sym_exec_hooks:
            hook()

    def execute_transactions(self, address) -> None:
        """svm.py:214-228: plugins may order transactions themselves
        (executed_transactions); otherwise transaction_count symbolic message
        calls."""
        for hook in self._start_exec_trans_hooks:
            hook()
        if self.executed_transactions is False:
            self._execute_transactions(address)
        for hook in self._stop_exec_trans_hooks:
            hook()

    def _execute_transactions(self, address) -> None:
        """svm.py:230-275: per transaction, the open states whose constraints
        are still possible (all queries of the round in one kernel-2 launch,
        answered in order), then one symbolic message call per open state."""
        from .transaction import execute_symbolic_message_call
        self.time = datetime.now()
        for _ in range(self.transaction_count):
            if len(self.open_states) == 0:
                break
            if self.use_reachability_check:
                self.open_states = self.reachable(self.open_states)
            for hook in self._start_sym_trans_hooks:
                hook()
            execute_symbolic_message_call(self, address)
            for hook in self._stop_sym_trans_hooks:
                hook()
        self.executed_transactions = True

    def reachable(self, world_states: list) -> list:
        """[ws for ws in world_states if ws.constraints.is_possible()] with the
        queries prefetched together (svm.py:244-249)."""
        self._flush_forks()
        if not world_states:
            return []
        kc = _keccak_conjunct()
        qs = [SnapshotConstraints(ws.constraints, kc) for ws in world_states]
        solver_mod.model_cache.prefetch([query_raw(q.get_all_constraints()) for q in qs])
        try:
            return [ws for ws, q in zip(world_states, qs) if self._possible(q)]
        finally:
            solver_mod.model_cache.clear_prefetch()

    def _host_only(self, states, final_states, track_gas):
        """States a lane cannot carry (a symbolic word the expression arena has
        no node for, symbolic storage or memory) take one step with the escape
        handler (the reference's execute_state) and come back through the work
        list; without a handler they are dropped as svm.py:314-316 drops a
        NotImplementedError.  Returns the lane-eligible states."""
        keep = []
        # the encodings made here serve the batch's _shape and _pack (one encode per state)
        self._pre_enc = pre = {}
        for st in states:
            le = sym.lane_encoding(st)
            if le is not None:
                keep.append(st)
                if le.symbolic:
                    pre[id(st)] = (st, le)
                continue
            self._flush_forks()
            if self.escape_handler is None:
                log.debug("state not representable on a lane and no escape handler: dropped")
                continue
            op = _opcode_at(st)
            new_states = self._escape_step(st, hooks_done=False, track_gas=track_gas,
                                           final_states=final_states)
            if new_states is None:
                continue
            self._filter_fork(new_states)
            self.manage_cfg(op, new_states)
            self.work_list.extend(new_states)
            self.total_states += len(new_states)
            if not new_states and track_gas:
                final_states.append(st)
        return keep

    def _escape_step(self, s: GlobalState, hooks_done: bool, track_gas: bool, final_states: list):
        """svm.py:369-491 execute_state for a state the escape handler steps.

        The handler is the instruction's mutator -- in an integration the
        reference's ``Instruction(op, dynamic_loader).evaluate(state)``: it
        returns the successor states or raises a transaction-end signal
        (``TransactionEndSignal``: ``global_state``, ``revert``), a VmException,
        a ``TransactionStartSignal`` or ``NotImplementedError``.  This method
        runs what execute_state runs around it: the execute_state hooks, the
        precheck, the svm and instruction pre hooks (unless the device already
        stopped the lane for them: ``hooks_done``), the transaction-end hooks,
        ``check_potential_issues`` and ``_add_world_state`` of a top-level end,
        and the post hooks on the successors.  Returns the successors, or None
        when the state was consumed without any (final states already noted)."""
        instrs = s.environment.code.instruction_list
        name = instrs[s.mstate.pc]["opcode"] if s.mstate.pc < len(instrs) else None
        if not hooks_done:
            try:
                for hook in self._execute_state_hooks:
                    hook(s)
            except PluginSkipState:
                if track_gas:
                    final_states.append(s)
                return None
            if name is None:
                self._add_world_state(s)                  # svm.py:384-389
                return None
            if len(s.mstate.stack) < get_required_stack_elements(name):
                if track_gas:                             # svm.py:391-402 precheck underflow
                    final_states.append(s)
                return None
            try:
                self._execute_pre_hook(name, s)
            except PluginSkipState:
                if track_gas:
                    final_states.append(s)
                return None
            for hook in self.instr_pre_hook.get(name, ()):
                hook(s)
        snapshot = copy(s) if self.instr_post_hook.get(name) else None
        try:
            new_states = list(self.escape_handler(s))
        except Exception as exc:          # noqa: BLE001 -- classified below, else re-raised
            kind = _signal_kind(exc)
            tx = s.current_transaction
            if kind == "end":
                self._end_transaction(exc.global_state, s, bool(getattr(exc, "revert", False)))
            elif kind == "vm":
                for hook in self._transaction_end_hooks:     # svm.py:417-425
                    hook(s, tx, None, False)
            elif kind in ("start", "unimplemented"):
                # svm.py:314-316: a NotImplementedError drops the path; a call
                # into code (a nested transaction) is outside the batched core
                log.debug("escape handler cannot step %s (%s): state dropped", name, type(exc).__name__)
                self.escapes_dropped += 1
            else:
                raise
            new_states = []
        if snapshot is not None:
            for hook in self.instr_post_hook.get(name, ()):
                hook(snapshot)
        if name is not None:
            self._execute_post_hook(name, new_states)
        return new_states

    def _end_transaction(self, end_state: GlobalState, pre_state: GlobalState, revert: bool) -> None:
        """svm.py:427-465 for a TransactionEndSignal: the transaction-end hooks;
        at the top level a kept end (not a revert, and a creation only when it
        returned code) runs check_potential_issues on the state before the
        ending instruction and adds the world state."""
        tx, return_state = end_state.transaction_stack[-1] if end_state.transaction_stack else (None, None)
        for hook in self._transaction_end_hooks:
            hook(end_state, tx, return_state, revert)
        if return_state is not None:
            log.debug("nested message call ends outside the batched core: state dropped")
            self.escapes_dropped += 1
            return
        if (not isinstance(tx, ContractCreationTransaction) or tx.return_data) and not revert:
            check_potential_issues(pre_state)
            end_state.world_state.node = pre_state.node
            self._add_world_state(end_state)

    def _filter_fork(self, new_states: list) -> None:
        """svm.py:319-326: a fork keeps the successors whose path constraints are
        possible (kernel-2 quick-sat over the model cache, then the backend)."""
        self._flush_forks()
        if self.strategy.run_check() and (len(new_states) > 1 and random.uniform(0, 1) < args.pruning_factor):
            new_states[:] = [st for st in new_states
                             if self._possible(Constraints(st.world_state.constraints))]

    def _possible(self, constraints) -> bool:
        self.fork_stats["queries"] += 1
        try:
            ok = constraints.is_possible()
        except SolverBackendMissing:
            if self.unknown_forks != "keep":
                raise
            self.fork_stats["unknown"] += 1
            ok = True
        self.fork_stats["kept" if ok else "pruned"] += 1
        return ok

    def _queue_fork(self, s: GlobalState, new_states: list, track_gas: bool, final_states: list) -> None:
        """svm.py:319-326 for an MG_FORK event, deferred: the decision to filter
        (and its random draw) and each successor's query -- the keccak conjunct
        as of now -- are taken here; the queries of consecutive forks are then
        evaluated together (_flush_forks) in the same order, so answers and
        model-cache moves are the sequential loop's."""
        queries = None
        if self.strategy.run_check() and (len(new_states) > 1 and random.uniform(0, 1) < args.pruning_factor):
            kc = _keccak_conjunct()
            queries = [SnapshotConstraints(st.world_state.constraints, kc) for st in new_states]
        self._pending_forks.append((s, new_states, queries, track_gas, final_states))

    def _flush_forks(self) -> None:
        pend = self._pending_forks
        if not pend:
            return
        self._pending_forks = []
        raws = [query_raw(q.get_all_constraints()) for _, _, qs, _, _ in pend if qs for q in qs]
        self.fork_stats["flushes"] += 1
        self.fork_stats["groups"] += len(pend)
        if raws:
            solver_mod.model_cache.prefetch(raws)
        try:
            for s, new_states, qs, track_gas, final_states in pend:
                if qs is not None:
                    new_states = [st for st, q in zip(new_states, qs) if self._possible(q)]
                self.work_list.extend(new_states)
                self.total_states += len(new_states)
                if not new_states and track_gas:
                    final_states.append(s)
        finally:
            solver_mod.model_cache.clear_prefetch()

    def manage_cfg(self, opcode: Optional[str], new_states: List[GlobalState],
                   parent: Optional[GlobalState] = None) -> None:
        """svm.py:549-573 for the successors a host step produced: a JUMP /
        JUMPI successor (and a RETURN's, i.e. the caller's state after a nested
        call) enters a new node, whose function name _new_node_state sets.
        Without requires_statespace only the name switch is kept; lanes apply
        it from the device's function-entry index (_materialise).  With it,
        _exec_stepwise calls this once per step (the calls inside that step are
        skipped) and the graph is built as the reference builds it."""
        if not self.requires_statespace:
            if opcode in ("JUMP", "JUMPI", "RETURN"):
                for state in new_states:
                    self._new_node_state(state)
            return
        if self._single_step:
            return
        if opcode == "JUMP":
            for state in new_states:
                self._new_graph_node(state)
        elif opcode == "JUMPI" or (opcode in ("SLOAD", "SSTORE") and len(new_states) > 1):
            for state in new_states:
                self._new_graph_node(state, JumpType.CONDITIONAL, self._edge_condition(state, parent))
        elif opcode == "RETURN":
            for state in new_states:
                self._new_graph_node(state, JumpType.RETURN)
        # a node keeps each state as of its instruction: the device path steps
        # the successor object itself onwards (materialised in place), where
        # the reference's StateTransition steps a copy, so the node gets one
        for state in new_states:
            if state.node is not None:
                state.node.states.append(copy(state))

    @staticmethod
    def _edge_condition(state: GlobalState, parent: Optional[GlobalState]):
        """state.world_state.constraints[-1] (svm.py:563): jumpi_ appends the
        simplified branch condition to every successor, True for a concrete one
        (instructions.py:1581-1631); a successor whose list did not grow took a
        concrete branch."""
        cons = state.world_state.constraints
        if parent is not None and len(cons) <= len(parent.world_state.constraints):
            return symbol_factory.Bool(True)
        return cons[-1] if len(cons) else None

    def _new_graph_node(self, state: GlobalState, edge_type=JumpType.UNCONDITIONAL,
                        condition=None) -> None:
        """svm.py:575-637: the successor enters a fresh node of its active
        account's contract, joined to its old node by an edge of `edge_type`;
        the function-name switch of _new_node_state, with FUNC_ENTRY set on the
        node where a dispatcher entry is entered."""
        env = state.environment
        code = env.code
        try:
            address = code.instruction_list[state.mstate.pc]["address"]
        except IndexError:
            return
        new_node = Node(env.active_account.contract_name)
        old_node = state.node
        state.node = new_node
        new_node.constraints = state.world_state.constraints
        self.nodes[new_node.uid] = new_node
        self.edges.append(Edge(old_node.uid if old_node is not None else None, new_node.uid,
                               edge_type=edge_type, condition=condition))
        if edge_type == JumpType.RETURN:
            new_node.flags |= NodeFlags.CALL_RETURN
        seq = state.world_state.transaction_sequence
        if seq and isinstance(seq[-1], ContractCreationTransaction):
            env.active_function_name = "constructor"
        elif address in code.address_to_function_name:
            env.active_function_name = code.address_to_function_name[address]
            new_node.flags |= NodeFlags.FUNC_ENTRY
        elif address == 0:
            env.active_function_name = "fallback"
        new_node.function_name = env.active_function_name

    def transaction_node(self, global_state: GlobalState, transaction) -> None:
        """transaction/symbolic.py:221-243 (concolic.py:134-156): a transaction's
        first state starts a node of the callee's contract, joined by a
        Transaction edge to the node its world state ended in."""
        if not self.requires_statespace:
            return
        env = global_state.environment
        new_node = Node(env.active_account.contract_name, function_name=env.active_function_name)
        self.nodes[new_node.uid] = new_node
        prev = transaction.world_state.node
        if prev is not None:
            self.edges.append(Edge(prev.uid, new_node.uid, edge_type=JumpType.Transaction,
                                   condition=None))
            new_node.constraints = global_state.world_state.constraints
        global_state.node = new_node
        new_node.states.append(copy(global_state))

    @staticmethod
    def _new_node_state(state: GlobalState) -> None:
        """svm.py:575-637, the environment part: a creation transaction's
        states are "constructor"; a successor at a dispatcher entry takes its
        name (Disassembly.address_to_function_name); at address 0, "fallback"."""
        env = state.environment
        code = env.code
        try:
            address = code.instruction_list[state.mstate.pc]["address"]
        except IndexError:
            return
        seq = state.world_state.transaction_sequence
        if seq and isinstance(seq[-1], ContractCreationTransaction):
            env.active_function_name = "constructor"
        elif address in code.address_to_function_name:
            env.active_function_name = code.address_to_function_name[address]
        elif address == 0:
            env.active_function_name = "fallback"

    def _apply_fent(self, b: LaneBatch, i: int, s: GlobalState) -> None:
        """The device's record of the lane's last JUMP / JUMPI landing on a
        function entry (mg_lane_soa.fent): _new_node_state at that successor --
        the last switch is the only one that shows (every switch overwrites the
        name; a landing elsewhere leaves it)."""
        fe = int(b.fent[i])
        if fe == MG_FENT_NONE:
            return
        env = s.environment
        seq = s.world_state.transaction_sequence
        if seq and isinstance(seq[-1], ContractCreationTransaction):
            env.active_function_name = "constructor"
            return
        name = env.code.name_at(fe)
        if name is not None:
            env.active_function_name = name

    def _add_world_state(self, global_state: GlobalState) -> None:
        """svm.py:339-348."""
        for hook in self._add_world_state_hooks:
            try:
                hook(global_state)
            except PluginSkipWorldState:
                return
        self.open_states.append(global_state.world_state)

    def execute_state(self, global_state: GlobalState) -> Tuple[List[GlobalState], Optional[str]]:
        """svm.py:369-491 for one state: a one-lane batch stepped one
        instruction on the device with the same hook protocol as exec()."""
        saved = self.work_list[:]
        del self.work_list[:]
        final: List[GlobalState] = []
        instrs = global_state.environment.code.instruction_list
        op = instrs[global_state.mstate.pc]["opcode"] if global_state.mstate.pc < len(instrs) else None
        self._single_step = True
        try:
            self._run_batch([global_state], final, False, True, single_step=True)
        finally:
            self._single_step = False
        successors = self.work_list[:]
        self.work_list[:] = saved
        return successors, op

    # ------------------------------------------------------------- hooks API
    def register_hooks(self, hook_type: str, hook_dict: Dict[str, List[Callable]]):
        if hook_type == "pre":
            entrypoint = self.pre_hooks
        elif hook_type == "post":
            entrypoint = self.post_hooks
        else:
            raise ValueError("Invalid hook type %s. Must be one of {pre, post}", hook_type)
        for op_code, funcs in hook_dict.items():
            entrypoint[op_code].extend(funcs)

    def register_laser_hooks(self, hook_type: str, hook: Callable):
        if hook_type in self.hook_type_map:
            self.hook_type_map[hook_type].append(hook)
        else:
            raise ValueError(f"Invalid hook type {hook_type}")

    def register_instr_hooks(self, hook_type: str, opcode: str, hook: Callable):
        table = self.instr_pre_hook if hook_type == "pre" else self.instr_post_hook
        if opcode is None:
            for op in OPCODES:
                table[op].append(hook(op))
        else:
            table[opcode].append(hook)

    def instr_hook(self, hook_type, opcode) -> Callable:
        def hook_decorator(func: Callable):
            self.register_instr_hooks(hook_type, opcode, func)
        return hook_decorator

    def laser_hook(self, hook_type: str) -> Callable:
        def hook_decorator(func: Callable):
            self.register_laser_hooks(hook_type, func)
            return func
        return hook_decorator

    def pre_hook(self, op_code: str) -> Callable:
        def hook_decorator(func: Callable):
            self.pre_hooks[op_code].append(func)
            return func
        return hook_decorator

    def post_hook(self, op_code: str) -> Callable:
        def hook_decorator(func: Callable):
            self.post_hooks[op_code].append(func)
            return func
        return hook_decorator

    def _execute_pre_hook(self, op_code: str, global_state: GlobalState) -> None:
        for hook in self.pre_hooks.get(op_code, ()):
            hook(global_state)

    def _execute_post_hook(self, op_code: str, global_states: List[GlobalState]) -> None:
        for hook in self.post_hooks.get(op_code, ()):
            for global_state in list(global_states):
                try:
                    hook(global_state)
                except PluginSkipState:
                    global_states.remove(global_state)

    def _hooked_ops(self):
        """Opcode bytes the device must stop before: any svm pre/post hook or
        instruction pre/post hook; all of them when execute_state hooks exist."""
        if self._execute_state_hooks:
            return set(range(256))
        ops = set()
        for table in (self.pre_hooks, self.post_hooks, self.instr_pre_hook, self.instr_post_hook):
            for name, hooks in table.items():
                if hooks and name in OPCODES:
                    ops.add(OPCODES[name])
        if self._plan is not None:
            ops -= self._plan.safe          # batch-safe hooks run on the device (laser/taint.py)
        return ops

    def _upload_force(self, dev) -> None:
        """mg_taint_force for every loaded code (laser/taint.py force_flags)."""
        for raw, cid in self._code_ids.items():
            dev.set_taint_force(cid, self._plan.force_flags(self._code_objs[raw]))

    def _annotators_registered(self) -> bool:
        """A module the taint registry knows (one whose hooks annotate words) is
        hooked, batch-safe or not: its annotate() calls need object identity."""
        for table in (self.pre_hooks, self.post_hooks):
            for hooks in table.values():
                for h in hooks:
                    m = tnt._module_of(h)
                    if m is not None and type(m).__name__ in tnt.BATCH_SAFE:
                        return True
        return False

    def _has_post(self, name: str) -> bool:
        return bool(self.post_hooks.get(name) or self.instr_post_hook.get(name)
                    or self._execute_state_hooks)

    # ------------------------------------------------------------- lanes
    def _shape(self, states: List[GlobalState], taint: bool = False) -> LaneShape:
        n = len(states)
        g = self._cap_grow
        msz = max((len(s.mstate.memory) for s in states), default=0)
        slots = max((s.environment.active_account.storage.n_entries() for s in states), default=0)
        cdl = max((len(s.environment.calldata) for s in states), default=0)    # 0 when symbolic
        trace_cap = 0
        if self._loop_bound():
            tl = max((len(_trace_of(s)) for s in states), default=0)
            trace_cap = max(4096 * g, 2 * tl)
        stack_cap = 1024 if n <= 4096 else min(1024, 128 * g)
        mem_cap = max(4096 * g, 2 * msz)
        mem_cap = min(mem_cap, max(1024, ((1 << 30) // max(n, 1)) // 32 * 32), 1 << 24)
        mem_cap = max(mem_cap, (msz + 31) // 32 * 32)
        mem_cap = (mem_cap + 31) // 32 * 32
        # symbolic lanes: their arena encodings (reused by _pack) size the planes
        self._encodings = {}
        pre, self._pre_enc = getattr(self, "_pre_enc", None) or {}, None
        n_nodes = n_consts = 0
        for s in states:
            got = pre.get(id(s))
            if got is not None and got[0] is s:
                le = self._encodings[id(s)] = got[1]
            elif sym.state_is_symbolic(s):
                le = self._encodings[id(s)] = sym.encode_state(s)
            else:
                continue
            n_nodes = max(n_nodes, len(le.enc.nodes))
            n_consts = max(n_consts, len(le.enc.consts))
        symbolic = bool(self._encodings)
        return LaneShape(n=n, stack_cap=stack_cap, mem_cap=mem_cap,
                         calldata_cap=max((cdl + 31) // 32 * 32, 32),
                         storage_cap=max(64 * g, 2 * slots + 16), trace_cap=trace_cap,
                         # taint lanes log a record per annotating / deferred hook: a
                         # log that fills escapes and regrows (a later batch, §7)
                         rec_cap=(4096 if taint else 512) * g,
                         node_cap=max(256 * g, 2 * n_nodes) if symbolic else 0,
                         const_cap=max(128 * g, 2 * n_consts) if symbolic else 0,
                         obj_cap=min(256 * g, 65536) if taint else 0)

    def _pack(self, b: LaneBatch, i: int, s: GlobalState) -> None:
        env, ms = s.environment, s.mstate
        tx = s.current_transaction
        gas_limit = getattr(tx, "gas_limit", None)
        b.code_id[i] = self.code_id(env.code)
        b.pc[i] = ms.pc
        sflags = 0
        le = None
        b.sp[i] = len(ms.stack)
        b.stack[i] = 0
        if b.symbolic:
            b.stag[i] = 0
            b.n_nodes[i] = b.n_consts[i] = 0
            b.mtag[i] = 0
            b.sttag[i] = 0
            le = self._encodings.pop(id(s), None) if getattr(self, "_encodings", None) else None
            if le is None:
                le = sym.encode_state(s, b.shape.node_cap, b.shape.const_cap)
            if le.symbolic:
                sflags = le.flags
                if self.dynamic_loader is None:
                    sflags |= MG_LANE_BALANCE        # BALANCE as an arena node (balance_ needs no loader)
            else:
                le = None
        # the terms behind the lane's first arena nodes, for _materialise's decode
        s._arena_prefix = le.enc.node_raw if le is not None else None
        if le is None:
            stack = [concrete(x) for x in ms.stack]
            if stack:
                b.stack[i, : len(stack)] = np.array(
                    [np.frombuffer(w.to_bytes(32, "little"), dtype="<u4") for w in stack])
        mem = ms.memory.raw()
        b.msize[i] = len(mem)
        b.memory[i] = 0
        b.memory[i, : len(mem)] = np.frombuffer(mem, dtype=np.uint8)
        b.depth[i] = ms.depth
        b.status[i] = MG_RUNNING
        b.aux[i] = 0
        b.flags[i] = (MG_LANE_STATIC if env.static else 0) | (
            MG_LANE_CREATION if isinstance(tx, ContractCreationTransaction) else 0) | sflags | (
            MG_LANE_RETDATA if s.last_return_data is not None else 0)
        b.gas_min[i] = ms.min_gas_used
        b.gas_max[i] = ms.max_gas_used
        b.gas_limit[i] = _NO_GAS_LIMIT if gas_limit is None else min(concrete(gas_limit), _NO_GAS_LIMIT)
        cd = env.calldata
        b.calldata[i] = 0
        if sym.is_symbolic_calldata(cd):
            b.calldata_len[i] = 0                   # MG_LANE_SYMCD: CALLDATA* make arena nodes
        else:
            b.calldata[i, : len(cd)] = np.frombuffer(cd, dtype=np.uint8)
            b.calldata_len[i] = len(cd)
        words = (env.address, env.sender, env.origin, env.callvalue, env.gasprice)
        for k in range(MG_ENV_WORDS):
            w = words[k]
            b.env[i, k] = 0 if (isinstance(w, Expression) and w.value is None) else word_to_limbs(concrete(w))
        if le is not None:
            le.write(b, i)            # stack, arena, memory tags and the storage chain
        else:
            slots = list(env.active_account.storage.slots().items())
            b.storage[i] = 0
            for k, (key, val) in enumerate(slots):
                b.storage[i, k, :8] = word_to_limbs(key)
                b.storage[i, k, 8:] = word_to_limbs(val)
            b.storage_count[i] = len(slots)
        b.ret_offset[i] = b.ret_len[i] = 0
        b.fent[i] = MG_FENT_NONE              # the host's environment holds the name so far
        if b.shape.trace_cap:
            tr = _trace_of(s)
            b.trace[i] = 0
            b.trace[i, : len(tr)] = tr
            b.trace_len[i] = len(tr)
        b.rec_len[i] = 0                # records already parsed into the replay queue
        if hasattr(b, "rec_seen"):
            b.rec_seen[i] = 0
        if b.taint:
            if tnt.pack(b, i, s, self._tl[i], self._plan):
                b.flags[i] |= MG_LANE_TAINT
            else:
                log.warning("state needs more than %d annotation atoms or objects: its lane drops "
                            "annotations", tnt.MAX_ATOMS)

    def _materialise(self, b: LaneBatch, i: int, s: GlobalState, fn: bool = True) -> GlobalState:
        """Write lane i of the host image back into its GlobalState (in place);
        with `fn`, the function-name switch of its last entry landing too
        (manage_cfg runs after a step's post hooks: callers that run post hooks
        on the successor apply it afterwards)."""
        if fn and not self._single_step:
            self._apply_fent(b, i, s)
        ms = s.mstate
        ms.pc = int(b.pc[i])
        sp = int(b.sp[i])
        symlane = b.symbolic and int(b.flags[i]) & MG_LANE_SYMBOLIC
        if symlane:
            stack, memory, storage = sym.decode_lane(b, i, s, getattr(s, "_arena_prefix", None))
            ms.stack = MachineStack(stack)
        elif b.taint and int(b.flags[i]) & MG_LANE_TAINT:
            ms.stack = MachineStack([symbol_factory.BitVecVal(w, 256) for w in rows_to_words(b.stack[i, :sp])])
        else:
            ms.stack = LazyStack(b.stack[i, :sp].tobytes())
        if b.taint and int(b.flags[i]) & MG_LANE_TAINT:
            ms.stack = MachineStack(tnt.materialise(b, i, s, self._tl[i], self._plan, list(ms.stack)))
        ms.depth = int(b.depth[i])
        ms.min_gas_used = int(b.gas_min[i])
        ms.max_gas_used = int(b.gas_max[i])
        acct = s.environment.active_account
        if symlane:
            # the lane's store chain and memory bytes (symbolic ones included)
            ms.memory = memory
            acct.storage = storage
        else:
            ms.memory = Memory(bytes(b.memory[i, : int(b.msize[i])]))
            acct.storage.set_slots_raw(b.storage[i, :int(b.storage_count[i])].tobytes())
        s.lane_steps = int(b.steps[i])
        if b.shape.trace_cap:
            ann = _annotation_of(s)
            ann.trace = [int(x) for x in b.trace[i, : int(b.trace_len[i])]]
        return s

    # ------------------------------------------------------------- function managers
    def _collect_records(self, b: LaneBatch, run: List[int]) -> None:
        """Queue the new function-manager records of lanes `run` (just downloaded)
        under their global execution key: (round, position) for BFS, (-position,
        round) for DFS -- the order in which the reference executes them."""
        if not b.shape.rec_cap:
            return
        for i in run:
            end, seen = int(b.rec_len[i]), int(b.rec_seen[i])
            if end <= seen:
                continue
            for r in b.records(i, seen):
                if r[1] == "symkeccak":
                    # the input as the lane's arena holds it now (its node is final)
                    r = (r[0], "symkeccak", sym.keccak_input(b, i, self._rec_lanes[i].state, r[2]))
                elif r[1] == "symexp":
                    r = (r[0], "symexp", sym.exp_operands(b, i, self._rec_lanes[i].state, r[2]))
                elif r[1] == "symlen":
                    r = (r[0], "symlen", sym.decode_node(b, i, self._rec_lanes[i].state, r[2]), r[3])
                key = (r[0], i) if self._rec_bfs else (-i, r[0])
                heapq.heappush(self._recq, (key, next(self._rec_seq), i, r))
            b.rec_seen[i] = end

    def _replay_records(self, lanes, bound=None, inclusive: bool = False) -> None:
        """Register the queued records with key < bound (<= when inclusive; all
        when bound is None): keccak_function_manager.create_keccak's
        concrete_hashes entry for each SHA3 (keccak_function_manager.py:95-114)
        and, for each EXP, exponent_function_manager's constraint appended to the
        path's constraints (instructions.py:624-638)."""
        q = self._recq
        while q and (bound is None or q[0][0] < bound or (inclusive and q[0][0] == bound)):
            _, _, i, r = heapq.heappop(q)
            if r[1] == "keccak":
                keccak_function_manager.register_concrete(r[2], r[3])
            elif r[1] == "symkeccak":
                keccak_function_manager.create_keccak(r[2])      # symbolic_inputs, in order
            elif r[1] == "annot":
                tnt.note_record(self._tl[i], r, lanes[i].state, self._plan)
            elif r[1] == "hook":
                tnt.replay_deferred(r, lanes[i].state, self._plan, self._tl[i])
            elif r[1] == "symexp":
                # exp_ of a symbolic operand (instructions.py:624-638): the manager's
                # condition on Power(base, exponent)
                _, cond = exponent_function_manager.create_condition(*r[2])
                lanes[i].state.world_state.constraints.append(cond)
            elif r[1] == "symlen":
                # sha3_ of a symbolic length (instructions.py:1023-1028): length 64
                lanes[i].state.world_state.constraints.append(r[2] == r[3])
            elif r[1] == "cdsize":
                # codesize_ of a creation (instructions.py:989-997): the symbolic
                # calldata's size is pinned to the pushed value
                st = lanes[i].state
                st.world_state.constraints.append(
                    st.environment.calldata.size == symbol_factory.BitVecVal(r[2], 256))
            else:
                _, cond = exponent_function_manager.create_condition(
                    symbol_factory.BitVecVal(r[2], 256), symbol_factory.BitVecVal(r[3], 256))
                lanes[i].state.world_state.constraints.append(cond)

    def _event_key(self, b: LaneBatch, i: int):
        r = _event_round(b, i)
        return (r, i) if self._rec_bfs else (-i, r)

    def _loop_bound(self) -> int:
        return int(getattr(self.strategy, "bound", 0) or 0)

    # ------------------------------------------------------------- the batch loop
    def _run_batch(self, states: List[GlobalState], final_states: List[GlobalState], create: bool,
                   track_gas: bool, single_step: bool = False):
        dev = self.device
        n = len(states)
        plan = tnt.TaintPlan(self)
        taint = (plan.active or self.track_objects or self._annotators_registered()
                 or any(tnt.state_needs_taint(s) for s in states))
        self._plan = plan if taint else None
        self._tl = [tnt.LaneTaint() for _ in states] if taint else None
        shape = self._shape(states, taint)
        b = LaneBatch(shape)
        b.rec_seen = np.zeros(n, dtype=np.int64)
        lanes = [_Lane(s, i) for i, s in enumerate(states)]
        for i, s in enumerate(states):
            self._pack(b, i, s)
            b.steps[i] = 0
        dev.alloc(shape, coverage=self.record_coverage)
        if taint:
            dev.set_taint_program(plan.actions)
            self._upload_force(dev)
        dev.upload(b)
        dev.set_loop_bound(self._loop_bound())
        mask = _mask(self._hooked_ops())
        plan_key = [plan.key()]
        depth = 0 if self.max_depth == _INF else int(self.max_depth)
        bfs = getattr(self.strategy, "order", "bfs") == "bfs"
        regrow: List[GlobalState] = []
        self._resumed = set()       # lanes a regrow resumed: not yet stepped (single_step)
        self._recq, self._rec_seq, self._rec_bfs, self._rec_lanes = [], itertools.count(), bfs, lanes

        sched = self._sched = _Schedule(lanes, b, bfs)

        def launch(run: List[int], horizon: int):
            # Between launches the host image equals the device image for every
            # lane that is not dirty (every lane the device may change is in
            # `run` and downloaded right after), so a copy may span clean lanes:
            # nearby ranges merge into one call (the fixed cost per call is far
            # above the per-lane bytes of a gap)
            for lo, cnt in _ranges(sorted(sched.dirty), gap=_MERGE_GAP):
                dev.upload_range(sched.b, lo, cnt, live=True)
                for pos in range(lo, lo + cnt):
                    lanes[pos].dirty = False
            sched.dirty.clear()
            if self._plan is not None and self._plan.key() != plan_key[0]:
                # a module's issue cache changed: its hooks may no longer be batch-safe
                self._plan = tnt.TaintPlan(self, prev=self._plan)
                plan_key[0] = self._plan.key()
                dev.set_taint_program(self._plan.actions)
                self._upload_force(dev)
                mask[:] = _mask(self._hooked_ops())
            st = dev.step(mask, max_steps=1 if single_step else (1 << 30), max_depth=depth,
                          horizon=horizon)
            self.launches += 1
            self._resumed.difference_update(run)
            self.device_ms += st.kernel_ms
            self.lane_steps += st.lane_steps
            self.total_states += st.lane_steps      # one successor per executed step
            for lo, cnt in _ranges(run, gap=_MERGE_GAP):
                dev.download_range(sched.b, lo, cnt, live=True)
            self._collect_records(sched.b, run)
            sched.set_after_launch(run)

        launch(list(range(n)), 0)
        try:
            return self._event_loop(b, lanes, sched, launch, final_states, create, track_gas, single_step, regrow)
        finally:
            self._flush_forks()

    def _event_loop(self, b, lanes, sched, launch, final_states, create, track_gas, single_step, regrow):
        bfs = sched.bfs
        while True:
            if (create and self._check_create_termination()) or (
                    not create and self._check_execution_termination()):
                self._replay_records(lanes)
                left = [self._materialise(b, ln.pos, ln.state) for ln in lanes
                        if ln.phase != "done"]
                return left
            ev = sched.next_event()
            if single_step:
                self._flush_forks()
                for i in sorted(sched.paused):
                    if i in self._resumed:
                        continue            # regrown before its step: launched below
                    ln = lanes[i]
                    self._materialise(b, i, ln.state)
                    self.work_list.append(ln.state)
                    sched.set(i, "done")
            if ev is None and not sched.paused:
                break
            if sched.paused:
                if bfs:
                    # paused paths might have events at or before ev's round
                    p_min = sched.paused_first()[0]
                    if ev is None or p_min <= _event_round(b, ev):
                        launch(sorted(sched.paused), 0 if ev is None else _event_round(b, ev) + 1)
                        continue
                elif ev is None or -sched.paused_first()[0] > ev:
                    launch(sorted(sched.paused), 0)     # DFS: the newest path runs on first
                    continue
            self._replay_records(lanes, self._event_key(b, ev))
            self._deliver(lanes[ev], b, final_states, track_gas, launch, regrow, single_step)
            if self._exec_stop:
                return None           # exec ends here: later events never happen
            if regrow:
                grown = self._regrow_in_place(b, regrow, lanes)
                if grown is not None:
                    b = sched.b = grown
                    regrow.clear()
        self._replay_records(lanes)
        self._flush_forks()
        if regrow:
            self._cap_grow *= 4
            self.work_list.extend(ln.state for ln, _ in regrow)
        return None

    def _deliver_plain_hook(self, ln: _Lane, b: LaneBatch, i: int, s: GlobalState, name: str, final_states,
                            track_gas, launch, regrow) -> None:
        """The MG_HOOK branch of _deliver for a plain concrete lane (its stack a
        LazyStack: no taint, symbolic or trace planes) with only pre hooks: the
        same steps (precheck, svm pre hooks, instruction pre hooks, copy if a hook
        kept the state, resume or repack, host halt, deferred launch), with the
        "hooks left the lane image alone" test reduced to the objects
        _materialise just made and the scalars it set."""
        ms, env = s.mstate, s.environment
        acct = env.active_account
        stack, mem, storage = ms.stack, ms.memory, acct.storage
        mver, sver = mem._ver, storage._ver
        scal = (ms.pc, ms.depth, ms.min_gas_used, ms.max_gas_used)
        ids = (id(env), id(acct), id(env.code), id(env.calldata), id(env.address), id(env.sender),
               id(env.origin), id(env.callvalue), id(env.gasprice), id(s.current_transaction), env.static)
        pre_state = s              # every local reference exists before the baseline counts
        refs0 = _held(s)
        if len(stack) < get_required_stack_elements(name):
            # svm.py:391-402: precheck underflow -- no pre hooks, no tx-end hooks
            if track_gas:
                final_states.append(s)
            return
        try:
            self._execute_pre_hook(name, s)
        except PluginSkipState:
            if track_gas:
                final_states.append(s)
            return
        for hook in self.instr_pre_hook.get(name, ()):
            hook(s)
        if self.always_copy_hooked or _held(s) != refs0:
            s = copy(s)                    # a hook kept the state: the lane goes on with a copy
            ln.state = s
        pm, pe = pre_state.mstate, pre_state.environment
        steps = int(b.steps[i])
        if (pm is ms and pm.stack is stack and not stack.mut and pm.memory is mem and mem._ver == mver
                and pe.active_account is acct and acct.storage is storage and storage._ver == sver
                and (pm.pc, pm.depth, pm.min_gas_used, pm.max_gas_used) == scal
                and (id(pe), id(pe.active_account), id(pe.code), id(pe.calldata), id(pe.address),
                     id(pe.sender), id(pe.origin), id(pe.callvalue), id(pe.gasprice),
                     id(pre_state.current_transaction), pe.static) == ids):
            _rearm(b, i)                   # the lane image is still the state's: only resume it
        else:
            self._pack(b, i, s)
            b.steps[i] = steps
        b.flags[i] |= MG_LANE_HOOK_ACK
        if self._halts_on_host(name, s, b, i):
            b.flags[i] = int(b.flags[i]) & ~MG_LANE_HOOK_ACK
            b.steps[i] = steps + 1
            self.lane_steps += 1
            self.total_states += 1
            self._sched.set(i, "event")
            self._deliver(ln, b, final_states, track_gas, launch, regrow, False)
            return
        sched = self._sched
        safe = sched.bfs and self._ack_safe(name, s, b)
        sched.set(i, "paused", acked=safe)
        sched.mark_dirty(i)

    def _regrow_in_place(self, b: LaneBatch, regrow, lanes) -> Optional[LaneBatch]:
        """A lane stopped by a full per-lane table (capacity escape): grow that
        capacity 4x for the whole batch, copy every lane into the new image
        (LaneBatch.regrown), re-allocate and re-upload, and resume the lane at the
        instruction it stopped before -- inside this batch, so its later events
        keep their place in the strategy's order and a hook it already passed is
        not run again.  None when the capacity is already at its limit (or the
        taint escape was the 64-atom limit): the caller re-queues the state for a
        later batch, where packing compacts it."""
        sh = b.shape
        grow = {}
        for ln, reason in regrow:
            need = _capacity_growth(sh, reason, b, ln.pos)
            if need is None:
                return None
            grow.update(need)
        if any(v <= getattr(sh, k) for k, v in grow.items()):
            return None
        # lanes of the same launch that escaped for a capacity this growth covers
        # resume too (their escape events are artifacts of the old shape)
        resume = [(ln.pos, reason) for ln, reason in regrow]
        for ln in lanes:
            i = ln.pos
            if ln.phase == "event" and int(b.status[i]) == MG_ESCAPE:
                need = _capacity_growth(sh, int(b.aux[i]) >> 8, b, i)
                if need and all(k in grow for k in need):
                    resume.append((i, int(b.aux[i]) >> 8))
        b2 = b.regrown(dataclasses.replace(sh, **grow))
        b2.rec_seen = b.rec_seen.copy()
        for i, reason in resume:
            b2.status[i] = MG_RUNNING
            b2.aux[i] = 0
            if reason != MG_ESC_TRACE and sh.trace_cap and int(b2.trace_len[i]):
                b2.trace_len[i] -= 1          # traced at its pop, traced again when it runs
        dev = self.device
        dev.alloc(b2.shape, coverage=self.record_coverage)
        if self._plan is not None:
            dev.set_taint_program(self._plan.actions)
            self._upload_force(dev)
        dev.upload(b2)
        dev.set_loop_bound(self._loop_bound())
        self.regrows += 1
        sched = self._sched
        for pos in sched.dirty:
            lanes[pos].dirty = False
        sched.dirty.clear()
        sched.b = b2
        for i, _ in resume:
            sched.set(i, "paused")
            self._resumed.add(i)
        return b2


    def _deliver(self, ln: _Lane, b: LaneBatch, final_states, track_gas, launch, regrow,
                 single_step: bool = False):
        """Run the host side of one device event, as execute_state would."""
        i, s = ln.pos, ln.state
        status = int(b.status[i])
        if status != MG_FORK:
            self._flush_forks()        # queued fork filters come first (reference order)
        self._materialise(b, i, s)
        if status == MG_FORK and len(s.mstate.stack) >= 2 and s.mstate.stack[-2].value is not None:
            # the device tagged the condition symbolic, but its term folds to a
            # constant on the host (an arena node over words the decode resolves:
            # a store-chain read, a memory read, a balance): the reference's JUMPI
            # is concrete there, so the lane takes the path of any instruction the
            # device left to the host -- exactly where a lane whose word was
            # concrete from the start goes (tests/oracle_device.py parks it so)
            self._flush_forks()
            status = MG_ESCAPE
            b.status[i] = MG_ESCAPE
            b.aux[i] = OPCODES["JUMPI"] | (MG_ESC_SYMBOLIC << 8)
        instrs = s.environment.code.instruction_list
        name = instrs[s.mstate.pc]["opcode"] if s.mstate.pc < len(instrs) else None
        self._sched.set(i, "done")
        if self.record_coverage and status in (MG_HOOK, MG_ESCAPE) and name is not None:
            self._host_cov[s.environment.code.raw].add(s.mstate.pc)

        if status in _EXECUTED_HALTS:
            self.total_states -= 1                  # the halting step had no successor
        if status == MG_HOOK and self._fast_hooks and type(s.mstate.stack) is LazyStack \
                and not self._execute_state_hooks \
                and not single_step and not self._has_post(name):
            self._deliver_plain_hook(ln, b, i, s, name, final_states, track_gas, launch, regrow)
            return
        if status == MG_HOOK:
            # plain concrete lanes: a state the hooks leave untouched needs no repack
            sig0 = _hook_sig(s) if not (b.taint or b.symbolic or b.shape.trace_cap) else None
            pre_state = s
            refs0 = _held(pre_state)
            # execute_state returning [] puts the popped state in final_states
            # when track_gas (svm.py:328-334), whatever the reason
            try:
                for hook in self._execute_state_hooks:
                    hook(s)
            except PluginSkipState:
                if track_gas:
                    final_states.append(s)
                return
            if len(s.mstate.stack) < get_required_stack_elements(name):
                # svm.py:391-402: precheck underflow -- no pre hooks, no tx-end hooks
                if track_gas:
                    final_states.append(s)
                return
            try:
                self._execute_pre_hook(name, s)
            except PluginSkipState:
                if track_gas:
                    final_states.append(s)
                return
            for hook in self.instr_pre_hook.get(name, ()):
                hook(s)
            post = self._has_post(name) or single_step
            # the hooks keep the state they saw (the reference's evaluate steps a
            # copy, instructions.py:121-130): the lane goes on with a copy -- unless
            # no hook kept a reference to the state or to any part of it the lane
            # changes later (_held), when nothing can observe the difference
            if post or self.always_copy_hooked or _held(pre_state) != refs0:
                s = copy(s)
                ln.state = s
            # hooks may have rewritten the state: repack, then run the hooked
            # instruction alone (STEP1) when post hooks must see its successor
            steps = int(b.steps[i])
            if sig0 is not None and sig0 == _hook_sig(pre_state):
                _rearm(b, i)             # the lane image is still the state's: only resume it
            else:
                self._pack(b, i, s)
            b.steps[i] = steps
            b.flags[i] |= MG_LANE_HOOK_ACK | (MG_LANE_STEP1 if post else 0)
            if not post and self._halts_on_host(name, s, b, i):
                # a hooked STOP / RETURN whose outcome is certain ends right here, as
                # the device would report it -- without a launch per such event
                b.flags[i] = int(b.flags[i]) & ~MG_LANE_HOOK_ACK
                b.steps[i] = steps + 1
                self.lane_steps += 1
                self.total_states += 1
                self._sched.set(i, "event")
                self._deliver(ln, b, final_states, track_gas, launch, regrow, single_step)
                return
            if not post:
                # BFS: a resumed instruction that cannot end, escape or register
                # at its own round joins the round's next launch instead of
                # forcing one before the round's later events (see _ack_safe)
                safe = self._sched.bfs and self._ack_safe(name, s, b)
                self._sched.set(i, "paused", acked=safe); self._sched.mark_dirty(i)
                return
            self._sched.mark_dirty(i)
            snapshot = copy(pre_state)
            launch([i], steps + 1)
            st2 = int(b.status[i])
            b.flags[i] = int(b.flags[i]) & ~(MG_LANE_HOOK_ACK | MG_LANE_STEP1) & 0xFFFFFFFF
            self._sched.mark_dirty(i)
            executed = int(b.steps[i]) == steps + 1
            if st2 in _EXECUTED_HALTS:
                if st2 == MG_HALT_DROPPED:
                    for hook in self.instr_post_hook.get(name, ()):
                        hook(snapshot)
                self._sched.set(i, "event")
                self._deliver(ln, b, final_states, track_gas, launch, regrow, single_step)
                return
            if not executed:      # escaped or cut by depth before running: its own event
                self._sched.set(i, "event")
                self._deliver(ln, b, final_states, track_gas, launch, regrow, single_step)
                return
            # the instruction's own registrations precede its post hooks
            self._replay_records(self._rec_lanes, (steps, i) if self._rec_bfs else (-i, steps),
                                 inclusive=True)
            for hook in self.instr_post_hook.get(name, ()):
                hook(snapshot)
            new = self._materialise(b, i, s, fn=False)
            successors = [new]
            self._execute_post_hook(name, successors)
            if not single_step:
                self._apply_fent(b, i, new)     # manage_cfg after the post hooks (svm.py:327)
            if not successors:
                self._sched.set(i, "done")
                if track_gas:
                    final_states.append(snapshot)
                return
            if st2 == MG_RUNNING:
                # post hooks may have rewritten the successor (an annotate() on
                # the pushed word, say): the lane resumes from the host image
                steps2 = int(b.steps[i])
                self._pack(b, i, new)
                b.steps[i] = steps2
                self._sched.mark_dirty(i)
            self._sched.set(i, "paused" if st2 == MG_RUNNING else "event")
            return

        tx = s.current_transaction
        if status in (MG_HALT_STOP, MG_HALT_RETURN):
            keep = True
            if isinstance(tx, ContractCreationTransaction):
                # transaction_models.py:265-284 + svm.py:459-466: only a creation
                # that returns code installs it and keeps its world state
                data = _return_data(b, i) if status == MG_HALT_RETURN else b""
                if data:
                    install_runtime_code(tx, s, data)
                else:
                    tx.return_data = None
                    keep = False
            elif status == MG_HALT_RETURN and tx is not None:
                tx.return_data = _return_data(b, i)
            for hook in self._transaction_end_hooks:
                hook(s, tx, None, False)
            if keep:
                check_potential_issues(s)                 # svm.py:456-462
                s.world_state.node = s.node
                self._add_world_state(s)
        elif status == MG_HALT_REVERT:
            if tx is not None:
                tx.return_data = _return_data(b, i)
            for hook in self._transaction_end_hooks:
                hook(s, tx, None, True)
        elif status == MG_HALT_END:
            if self._loop_bound():
                # BoundedLoopsStrategy.get_strategic_global_state reads the popped
                # state's current instruction: past the end that IndexError ends the
                # strategy's iteration (StopIteration), i.e. the whole exec, and this
                # state is never executed (bounded_loops.py:103-145, strategy/__init__.py)
                self._exec_stop = True
                return
            self._add_world_state(s)
        elif status == MG_VMEXC:
            precheck = (int(b.aux[i]) == MG_EXC_STACK_UNDERFLOW and name is not None
                        and len(s.mstate.stack) < get_required_stack_elements(name))
            if not precheck:
                for hook in self._transaction_end_hooks:
                    hook(s, tx, None, False)
        elif status == MG_HALT_DROPPED:
            pass
        elif status in (MG_DEPTH, MG_LOOP_BOUND):
            return                  # the strategy skips it: not a final state
        elif status == MG_FORK:
            # instructions.py:1558-1636 on a symbolic condition, then the fork
            # filter of svm.py:319-326 (kernel 2)
            self.forks += 1
            if self._plan is not None and OPCODES["JUMPI"] in self._plan.safe:
                # the device stops before a symbolic JUMPI without its batch-safe
                # pre-hooks: the reference runs them before the fork
                try:
                    self._execute_pre_hook("JUMPI", s)
                except PluginSkipState:
                    if track_gas:
                        final_states.append(s)
                    return
            successors = sym.jumpi_successors(s)
            self.manage_cfg("JUMPI", successors)     # the filter only drops states: same names
            self._queue_fork(s, successors, track_gas, final_states)
            return
        elif status == MG_ESCAPE:
            reason = int(b.aux[i]) >> 8
            if reason in (MG_ESC_MEMORY, MG_ESC_STORAGE, MG_ESC_STACK, MG_ESC_TRACE, MG_ESC_RECORD,
                          MG_ESC_ARENA, MG_ESC_TAINT):
                # rerun with larger lane capacities; the instruction was traced
                # at its pop but not executed, and will be traced again
                if reason != MG_ESC_TRACE and b.shape.trace_cap:
                    ann = _annotation_of(s)
                    if ann.trace:
                        ann.trace.pop()
                regrow.append((ln, reason))
                return
            if self.escape_handler is None:
                log.debug("Encountered unimplemented instruction %s", name)
                self.escapes_dropped += 1
                return              # svm.py:314-316: NotImplementedError -> continue
            # the device stopped the lane for this instruction's pre hooks first
            # (hook mask), so they have run -- unless they are batch-safe device
            # actions (laser/taint.py), which an escaping instruction never applied
            batch_safe = (self._plan is not None and name is not None
                          and OPCODES.get(name) in self._plan.safe)
            new_states = self._escape_step(s, hooks_done=not batch_safe, track_gas=track_gas,
                                           final_states=final_states)
            if new_states is None:
                return
            self._filter_fork(new_states)
            self.manage_cfg(name, new_states)
            self.work_list.extend(new_states)
            self.total_states += len(new_states)
            if new_states or not track_gas:
                return
        if track_gas:
            final_states.append(s)


    def _halts_on_host(self, name: str, s: GlobalState, b: LaneBatch, i: int) -> bool:
        """Set lane i's halt for a hooked STOP, or a RETURN that needs no memory
        extension and cannot run out of gas, exactly as kernel 1 would report it
        (instructions.py:1857-1959: STOP ends before any gas check; RETURN's
        mem_extend and check_gas_usage_limit, :1864-1872, change nothing here).
        False when the outcome needs the device."""
        if name == "STOP":
            b.status[i] = MG_HALT_STOP
            return True
        if name != "RETURN":
            return False
        st = s.mstate.stack
        if len(st) < 2:
            return False
        off, ln = st[-1].value, st[-2].value
        if off is None or ln is None or off + ln >= 1 << 32:
            return False
        msize = len(s.mstate.memory)
        if (ln == 0 and off > msize) or (ln and off + ln > msize):
            return False                       # mem_extend would extend (and charge gas)
        tx = s.current_transaction
        lim = getattr(tx, "gas_limit", None)
        lim = None if lim is None else (lim.value if isinstance(lim, Expression) else int(lim))
        gmin = s.mstate.min_gas_used
        if lim is None or gmin >= lim or gmin > 10 ** 9 or s.mstate.max_gas_used > 10 ** 9:
            return False
        b.status[i] = MG_HALT_RETURN
        b.ret_offset[i], b.ret_len[i] = off, ln
        return True

    def _ack_safe(self, name: str, s: GlobalState, b: LaneBatch) -> bool:
        """True when the hooked instruction of `s`, resumed with HOOK_ACK, can
        produce no event and no function-manager record at its own round: no
        halt, VmException, dropped jump, capacity or opcode escape, OOG.  Under
        BFS the reference runs it right after its hooks (svm.py:369-491) and the
        next event of the same round comes after it; when it can affect nothing
        that event sees, the launch that executes it can wait until the round's
        events are delivered, so one launch serves the whole round.  The test
        is conservative: any doubt answers False (launch now, as before)."""
        real_pops = _ACK_SAFE.get(name)
        if real_pops is None:
            return False
        ms, env = s.mstate, s.environment
        st = ms.stack
        n = len(st)
        if n < real_pops:
            return False                 # the real pop raises (table counts differ)
        if type(st) is LazyStack:
            top = st.top_int             # a concrete lane's words, read without building them
        else:
            if real_pops and any(isinstance(x, Expression) and x.value is None for x in st[-real_pops:]):
                return False             # symbolic operand: a fork or escape at this round

            def top(k):
                return concrete(st[-k])
        if (name.startswith("PUSH") or name.startswith("DUP")) and n + 1 > min(1024, b.shape.stack_cap):
            return False
        extra = 0
        if name in ("MLOAD", "MSTORE", "MSTORE8"):
            off = top(1)
            end = off + (1 if name == "MSTORE8" else 32)
            if end > b.shape.mem_cap:
                return False             # capacity escape
            w = (end + 31) // 32
            extra = 3 * w + w * w // 512
        elif name == "SSTORE":
            if env.static:
                return False
            store = env.active_account.storage.printable_storage
            if top(1) not in store and len(store) >= b.shape.storage_cap:
                return False
        elif name in ("JUMP", "JUMPI"):
            if name == "JUMPI" and top(2) == 0:
                pass
            elif not self._jumpdest_at(env.code, top(1)):
                return False             # VmException / dropped branch at this round
        tx = s.current_transaction
        lim = getattr(tx, "gas_limit", None)
        lim = 10 ** 9 if lim is None else min(concrete(lim), 10 ** 9)
        # 50,000 bounds every listed opcode's table gas (SSTORE 20,000 at most)
        return ms.min_gas_used + extra + 50_000 < lim

    def _jumpdest_at(self, code, target: int) -> bool:
        """instructions.py:1520-1636 jump check: the first instruction at or above
        `target` (util.get_instruction_index's >=) is a JUMPDEST."""
        key = code.bytecode
        addrs = self._jd_addrs.get(key)
        if addrs is None:
            addrs = self._jd_addrs[key] = [ins["address"] for ins in code.instruction_list]
        if not addrs or target > addrs[-1]:
            return False
        k = bisect.bisect_left(addrs, target)
        return code.instruction_list[k]["opcode"] == "JUMPDEST"

    # ------------------------------------------------------------- coverage
    def coverage(self) -> Dict[object, Tuple[int, List[bool]]]:
        """coverage_plugin.py's table {bytecode: (n_instructions, [covered])} from
        the device's per-code coverage bytes (plus host-recorded marks)."""
        out = {}
        for raw, cid in self._code_ids.items():
            bits = self.device.coverage(cid).astype(bool)
            for pc in self._host_cov.get(raw, ()):
                if pc < bits.size:
                    bits[pc] = True
            peer = self._peer_cov.get(self._code_objs[raw].bytecode)
            if peer is not None:
                bits[:min(bits.size, peer.size)] |= peer[:bits.size].astype(bool)
            out[self._code_objs[raw].bytecode] = (int(bits.size), bits.tolist())
        for code, peer in self._peer_cov.items():
            if code not in out:
                out[code] = (int(peer.size), peer.astype(bool).tolist())
        return out

    def merge_peer_coverage(self, table: Dict[str, np.ndarray]) -> None:
        """OR other ranks' coverage bytes ({bytecode: uint8[n]}) into coverage()."""
        for code, bits in table.items():
            bits = np.asarray(bits, dtype=np.uint8)
            old = self._peer_cov.get(code)
            if old is not None and old.size == bits.size:
                bits = old | bits
            self._peer_cov[code] = bits


_KC = [None, None]


def _keccak_conjunct():
    """keccak_function_manager.create_conditions(), rebuilt only when an input
    or a hash was registered since the last call (it depends on nothing else:
    the intervals are assigned once per input size)."""
    km = keccak_function_manager
    def key():
        return (id(km), id(km.symbolic_inputs), id(km.concrete_hashes),
                tuple(len(v) for v in km.symbolic_inputs.values()), len(km.concrete_hashes),
                len(km.interval_hook_for_size))
    if _KC[0] != key():
        _KC[1] = km.create_conditions()
        _KC[0] = key()            # after the call: it may assign intervals
    return _KC[1]


def _annotation_of(state: GlobalState) -> JumpdestCountAnnotation:
    for a in state.annotations:
        if isinstance(a, JumpdestCountAnnotation):
            return a
    a = JumpdestCountAnnotation()
    state.annotate(a)
    return a


def _trace_of(state: GlobalState) -> List[int]:
    for a in state.annotations:
        if isinstance(a, JumpdestCountAnnotation):
            return a.trace
    return []


def _hook_sig(s: GlobalState):
    """What _pack reads from a concrete state, by identity and mutation count:
    equal before and after the hooks means the lane image is still the state's."""
    ms, env = s.mstate, s.environment
    acct = env.active_account
    stack = ms.stack
    # a lane's LazyStack records its own changes: no element is built to compare
    st = (stack.mut,) if type(stack) is LazyStack else (len(stack), tuple(map(id, stack)))
    return (ms.pc, id(stack), st, id(ms.memory), ms.memory._ver,
            ms.depth, ms.min_gas_used, ms.max_gas_used, id(env), id(env.code), env.static, id(env.calldata),
            id(env.address), id(env.sender), id(env.origin), id(env.callvalue), id(env.gasprice),
            id(acct), id(acct.storage), acct.storage._ver, id(s.current_transaction))


def _opcode_at(state: GlobalState) -> Optional[str]:
    instrs = state.environment.code.instruction_list
    pc = state.mstate.pc
    return instrs[pc]["opcode"] if pc < len(instrs) else None


def _no_potential_issues(state: GlobalState) -> None:
    """Default of the check_potential_issues seam: no analysis installed."""


# svm.py:456-462 calls mythril.analysis.potential_issues.check_potential_issues
# at every kept top-level transaction end; an integration installs it here
# (``mythril_amd.laser.svm.check_potential_issues = check_potential_issues``)
check_potential_issues: Callable[[GlobalState], None] = _no_potential_issues


def _signal_kind(exc: BaseException) -> Optional[str]:
    """What an escape handler's exception means to execute_state, by the
    reference's class names (so its own Instruction.evaluate can be the
    handler): a transaction end, a VmException, a nested transaction start, an
    unimplemented opcode; None for anything else (a real error)."""
    names = {k.__name__ for k in type(exc).__mro__}
    if "TransactionEndSignal" in names:
        return "end"
    if "VmException" in names:
        return "vm"
    if "TransactionStartSignal" in names:
        return "start"
    if "NotImplementedError" in names:
        return "unimplemented"
    return None


def _held(s: GlobalState) -> Tuple[int, ...]:
    """Reference counts of a state and of the parts of it a lane's next
    materialisation or host step changes in place (machine state, world state,
    its constraint and annotation lists, the environment, the active account and
    its storage, the transaction stack, the annotations): equal before and after
    the hooks means no hook kept any of them."""
    ws, env = s.world_state, s.environment
    acct = env.active_account
    ms = s.mstate
    rc = sys.getrefcount
    out = (rc(s), rc(ms), rc(ms.stack), rc(ms.memory), rc(ws), rc(ws.constraints), rc(ws._annotations),
           rc(env), rc(acct), rc(acct.storage), rc(s.transaction_stack), rc(s._annotations))
    if s._annotations:
        out += tuple(rc(a) for a in s._annotations)
    return out


def _rearm(b: LaneBatch, i: int) -> None:
    """The per-launch fields _pack resets, for a lane whose image is unchanged."""
    b.status[i] = MG_RUNNING
    b.aux[i] = 0
    b.flags[i] = int(b.flags[i]) & ~(MG_LANE_HOOK_ACK | MG_LANE_STEP1) & 0xFFFFFFFF
    b.ret_offset[i] = b.ret_len[i] = 0
    b.rec_len[i] = 0
    if hasattr(b, "rec_seen"):
        b.rec_seen[i] = 0


def _mask(ops) -> List[int]:
    m = [0, 0, 0, 0]
    for o in ops:
        m[o >> 6] |= 1 << (o & 63)
    return m


def _ranges(idx: List[int], gap: int = 0):
    """[first, count] runs covering the sorted lane indices; runs whose gap is
    at most `gap` lanes merge (the gap lanes are copied too)."""
    idx = sorted(idx)
    out = []
    for i in idx:
        if out and out[-1][0] + out[-1][1] + gap >= i:
            out[-1][1] = i - out[-1][0] + 1
        else:
            out.append([i, 1])
    return out


def _event_round(b: LaneBatch, i: int) -> int:
    st = int(b.status[i])
    s = int(b.steps[i])
    return s - 1 if st in _EXECUTED_HALTS else s

def _capacity_growth(sh: LaneShape, reason: int, b: LaneBatch, i: int) -> Optional[Dict[str, int]]:
    """The capacities (4x) a lane's capacity escape asks for; None when growing
    cannot help (the 64-atom limit of a taint lane) or it is no capacity escape."""
    n = sh.n
    if reason == MG_ESC_MEMORY:
        cap = min(sh.mem_cap * 4, max(1024, ((1 << 30) // max(n, 1)) // 32 * 32), 1 << 24)
        return {"mem_cap": (cap + 31) // 32 * 32}
    if reason == MG_ESC_STORAGE:
        return {"storage_cap": sh.storage_cap * 4}
    if reason == MG_ESC_STACK:
        return {"stack_cap": min(MG_STACK_LIMIT, sh.stack_cap * 4)}
    if reason == MG_ESC_TRACE:
        return {"trace_cap": sh.trace_cap * 4}
    if reason == MG_ESC_RECORD:
        return {"rec_cap": sh.rec_cap * 4}
    if reason == MG_ESC_ARENA:
        return {"node_cap": sh.node_cap * 4, "const_cap": sh.const_cap * 4}
    if reason == MG_ESC_TAINT and sh.obj_cap and sh.obj_cap < 65536 and (
            int(b.n_obj[i]) + 4 > sh.obj_cap or int(b.n_atoms[i]) + 2 <= 64):
        # the object table was full (a lane escapes for it after compacting, so
        # its stored count may be below the cap), not the 64-atom limit
        return {"obj_cap": min(sh.obj_cap * 4, 65536)}
    return None


class _Schedule:
    """Phases of one batch's lanes with O(log n) access to what the event loop
    needs: the next event in the reference's order (BFS: smallest (round,
    position); DFS: (-position, round)), the paused lanes (BFS: fewest
    cumulative steps first; DFS: highest position first) and the lanes whose
    host image changed.  Heaps with lazy deletion: an entry is valid while its
    lane is still in that phase with the same key."""

    def __init__(self, lanes: List[_Lane], b: LaneBatch, bfs: bool):
        self.lanes, self.b, self.bfs = lanes, b, bfs
        self._ev: List = []
        self._pz: List = []           # DFS: (-pos,) heap of paused lanes, lazy deletion
        # BFS: only the smallest paused round is ever asked for, so paused lanes
        # are counted per round (steps + acked) with a heap of the rounds: a
        # launch of thousands of lanes costs one count per lane, not one heap entry
        self._pround: Dict[int, int] = {}      # paused pos -> its round
        self._pcount: Dict[int, int] = {}      # round -> paused lanes
        self._prounds: List[int] = []          # heap of rounds (lazy: zero counts popped)
        self.paused: set = set()
        self.acked: set = set()       # paused at a deferred hooked instruction (_ack_safe)
        self.dirty: set = set()

    def _key(self, pos: int):
        r = _event_round(self.b, pos)
        return (r, pos) if self.bfs else (-pos, r)

    def _punpause(self, pos: int) -> None:
        r = self._pround.pop(pos, None)
        if r is not None:
            self._pcount[r] -= 1

    def _ppause(self, pos: int, r: int) -> None:
        self._pround[pos] = r
        c = self._pcount.get(r, 0)
        if not c:
            heapq.heappush(self._prounds, r)
        self._pcount[r] = c + 1

    def set(self, pos: int, phase: str, acked: bool = False) -> None:
        self.lanes[pos].phase = phase
        if self.bfs:
            self._punpause(pos)
        self.paused.discard(pos)
        self.acked.discard(pos)
        if phase == "event":
            heapq.heappush(self._ev, (self._key(pos), pos))
        elif phase == "paused":
            self.paused.add(pos)
            if acked:
                self.acked.add(pos)
            if self.bfs:
                # a deferred hooked instruction has no event before the next round
                self._ppause(pos, int(self.b.steps[pos]) + (1 if acked else 0))
            else:
                heapq.heappush(self._pz, ((-pos,), pos))

    def set_after_launch(self, run: List[int]) -> None:
        """set(i, "paused" | "event") for every lane of a launch, from one vector
        read of their status and steps (the per-lane form cost ~2 us a lane)."""
        idx = np.asarray(run, dtype=np.int64)
        st = self.b.status[idx]
        steps = self.b.steps[idx]
        running = st == MG_RUNNING
        run_p, steps_p = idx[running].tolist(), steps[running].tolist()
        run_e, st_e, steps_e = idx[~running].tolist(), st[~running].tolist(), steps[~running].tolist()
        lanes, paused, acked, bfs = self.lanes, self.paused, self.acked, self.bfs
        ev, push = self._ev, heapq.heappush
        acked.difference_update(run)
        paused.difference_update(run_e)
        paused.update(run_p)
        if bfs:
            # every lane of the launch leaves its paused round; the running ones
            # join their new round (counts in bulk)
            pround, pcount = self._pround, self._pcount
            for r in (pround.pop(i, None) for i in run):
                if r is not None:
                    pcount[r] -= 1
            for r, c in Counter(steps_p).items():
                old = pcount.get(r, 0)
                if not old:
                    push(self._prounds, r)
                pcount[r] = old + c
            pround.update(zip(run_p, steps_p))
        else:
            pz = self._pz
            for i in run_p:
                push(pz, ((-i,), i))
        for i in run_p:
            lanes[i].phase = "paused"
        for i, s_, k_ in zip(run_e, st_e, steps_e):
            lanes[i].phase = "event"
            r = k_ - 1 if s_ in _EXECUTED_HALTS else k_
            push(ev, ((r, i) if bfs else (-i, r), i))

    def mark_dirty(self, pos: int) -> None:
        self.lanes[pos].dirty = True
        self.dirty.add(pos)

    def next_event(self) -> Optional[int]:
        while self._ev:
            key, pos = self._ev[0]
            if self.lanes[pos].phase == "event" and key == self._key(pos):
                return pos
            heapq.heappop(self._ev)
        return None

    def paused_first(self):
        """Key of the first paused lane: (round,) under BFS (its cumulative steps,
        + 1 at a deferred hooked instruction), (-pos,) under DFS."""
        if self.bfs:
            h, cnt = self._prounds, self._pcount
            while h:
                if cnt.get(h[0]):
                    return (h[0],)
                heapq.heappop(h)
            return None
        while self._pz:
            key, pos = self._pz[0]
            if pos in self.paused and key == (-pos,):
                return key
            heapq.heappop(self._pz)
        return None


def _next_event(lanes: List[_Lane], b: LaneBatch, bfs: bool) -> Optional[int]:
    best, key = None, None
    for ln in lanes:
        if ln.phase != "event":
            continue
        r = _event_round(b, ln.pos)
        k = (r, ln.pos) if bfs else (-ln.pos, r)
        if key is None or k < key:
            best, key = ln.pos, k
    return best


def _return_data(b: LaneBatch, i: int) -> bytes:
    return b.return_data(i)
