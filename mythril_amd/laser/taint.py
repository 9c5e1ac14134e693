"""Annotation (taint) handles on the device and batch-safe hooks — SURVEY §8(f)1.

In the reference every stack word is a Python object with a mutable set of
annotations (laser/smt/expression.py:10-57).  ALU results take the union of
their operands' sets (bitvec.py:63-136, bitvec_helper.py), DUP pushes the same
object again (instructions.py:330), the environment words are one object each
(instructions.py:895-1060), and concrete memory and storage round trips drop the
sets (memory.py:84-115, account.py:43-87, array.py:21-28).  Detection modules
build on that: the integer module's ADD/SUB/MUL/EXP pre-hooks ``annotate()`` the
first operand with an ``OverUnderflowAnnotation`` and its SSTORE/JUMPI pre-hooks
collect the annotations that reach them into a state annotation
(analysis/module/modules/integer.py:133-260); TxOrigin annotates ORIGIN's word
and inspects JUMPI conditions (dependence_on_origin.py:44-107).

A taint lane (MG_LANE_TAINT, include/mythgpu.h) carries that object graph on
the device: an object handle per stack slot and an annotation mask per object
over up to 64 *atoms*, each atom one host-side set of annotation objects.  This
module is the host half:

* ``BATCH_SAFE``: the reference modules whose hooks the device reproduces, and
  how (Annotate / AnnotateResult / Sink / YieldIf).  ``TaintPlan`` turns the
  hooks a LaserEVM has registered into the device's per-opcode action words and
  the set of opcodes that no longer need to stop the lane;
* ``LaneTaint``: per lane, handle -> Python object and atom -> annotation set;
  ``pack`` writes a state's objects into the planes, ``materialise`` rebuilds
  them (the same Python objects where they existed, so identity and in-place
  annotation behave as in the reference);
* the device logs an MG_REC_ANNOT record for every atom it creates; when the
  host replays the lane's records in the reference's global order it runs the
  module's *own* hook (``module.execute``) on a state built from the record, and
  the annotations the hook adds become the atom's set.  A sink hook is replayed once per
  materialisation on the lane's real state with a word carrying everything the
  sinks collected, so the module's own state annotation receives them.

A cached issue address makes DetectionModule.execute return early there
(base.py:79-86): the device stops lanes at those instructions (mg_taint_force)
and the host runs the hooks.
"""
from __future__ import annotations

from collections import Counter
from copy import copy
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from ..lanes import (MG_TAINT_CDSIZE, MG_TAINT_DEFER_SHIFT, MG_TAINT_EXPCOND, MG_TAINT_IFLANE,
                     MG_TAINT_IFSYM_SHIFT, MG_TAINT_OBJ0, MG_TAINT_POST, MG_TAINT_SINK_SHIFT, MG_TAINT_YCLASS,
                     MG_TAINT_YIELD_SHIFT)
from ..smt.expr import Expression, symbol_factory
from .opcodes import OPCODES

MAX_ATOMS = 64
_ENV_ATTRS = ("address", "sender", "origin", "callvalue", "gasprice")     # handles 1..5 (MG_ENV_k + 1)


@dataclass(frozen=True)
class Annotate:
    """A pre-hook that annotate()s stack[-1-operand] (0 or 1); exp_cond: the
    integer module's EXP early return (integer.py:161-166)."""
    operand: int = 0
    exp_cond: bool = False
    yield_class: bool = False


@dataclass(frozen=True)
class AnnotateResult:
    """A post-hook that annotate()s the word the opcode pushed."""
    yield_class: bool = False


@dataclass(frozen=True)
class Sink:
    """A pre-hook that adds stack[-1-operand]'s annotations to a state annotation."""
    operand: int


@dataclass(frozen=True)
class YieldIf:
    """A pre-hook with work only when stack[-1-operand] carries an annotation of
    one of `types` (class names in the module's own Python module)."""
    operand: int
    types: Tuple[str, ...]


@dataclass(frozen=True)
class Deferred:
    """A pre-hook that changes nothing the path executes (it files issues or
    updates state annotations) and reads only stack[-1..-words], the pc, the
    environment and the path constraints: the device logs those words
    (MG_REC_HOOK) and the host runs the hook on them when it replays the lane's
    records, in the reference's order."""
    words: int = 1


@dataclass(frozen=True)
class IfSymbolic:
    """A pre-hook with work only when stack[-1-operand] is symbolic."""
    operand: int


@dataclass(frozen=True)
class IfStateAnnotation:
    """A pre-hook with work only when the state carries an annotation of one of
    `types`, or lacks one of `missing` (class names in the module's Python
    module); such annotations come from host events, so the host knows them
    when it packs the lane.  `missing`: StateChangeAfterCall's hook
    (state_change_external_calls.py:124-131) creates an empty
    PotentialIssuesAnnotation on a state that has none, even when it files
    nothing -- and that matters: the annotation has no __copy__, so every
    state copied from this one later shares its issue list
    (potential_issues.py:65-90), and a potential issue one branch files is
    checked at the other branch's transaction end.  So the device stops there
    (the host runs the hook) until the state has one."""
    types: Tuple[str, ...]
    missing: Tuple[str, ...] = ()


# The reference's modules (class name) -> {(hook type, opcode): action}
BATCH_SAFE: Dict[str, Dict[Tuple[str, str], object]] = {
    # analysis/module/modules/integer.py:75-85, 140-250
    "IntegerArithmetics": {
        ("pre", "ADD"): Annotate(0), ("pre", "MUL"): Annotate(0), ("pre", "SUB"): Annotate(0),
        ("pre", "EXP"): Annotate(0, exp_cond=True),
        ("pre", "SSTORE"): Sink(1), ("pre", "JUMPI"): Sink(1),
    },
    # analysis/module/modules/dependence_on_origin.py:33-34, 53-107
    "TxOrigin": {
        ("post", "ORIGIN"): AnnotateResult(yield_class=True),
        ("pre", "JUMPI"): YieldIf(1, ("TxOriginAnnotation",)),
    },
    # dependence_on_predictable_vars.py:47-48, 66-75: JUMPI has work only on a
    # PredictableValueAnnotation (its block-value post hooks run on the host:
    # those opcodes escape the device anyway)
    "PredictableVariables": {("pre", "JUMPI"): YieldIf(1, ("PredictableValueAnnotation",))},
    # arbitrary_jump.py:50, 74-77: a concrete target returns at once
    "ArbitraryJump": {("pre", "JUMP"): IfSymbolic(0), ("pre", "JUMPI"): IfSymbolic(0)},
    # arbitrary_write.py:28, 37-75: every SSTORE files a potential issue on the
    # state's PotentialIssuesAnnotation from the slot, pc and constraints
    "ArbitraryStorage": {("pre", "SSTORE"): Deferred(1)},
    # user_assertions.py:38, 55-64: MSTORE reads only the stored value (LOG1 reads
    # memory: a host hook)
    "UserAssertions": {("pre", "MSTORE"): Deferred(2)},
    # exceptions.py:43, 66-82: JUMP records its address in the LastJumpAnnotation
    "Exceptions": {("pre", "JUMP"): Deferred(1)},
    # state_change_external_calls.py:112, 148-160: SLOAD/SSTORE return at once
    # while the state has no StateChangeCallsAnnotation (made by CALL hooks)
    "StateChangeAfterCall": {("pre", "SLOAD"): IfStateAnnotation(("StateChangeCallsAnnotation",),
                                                                 ("PotentialIssuesAnnotation",)),
                             ("pre", "SSTORE"): IfStateAnnotation(("StateChangeCallsAnnotation",),
                                                                  ("PotentialIssuesAnnotation",))},
}


def register_batch_safe(module_class_name: str, table: Dict[Tuple[str, str], object]) -> None:
    """Declare another module's hooks batch-safe (same action vocabulary)."""
    BATCH_SAFE[module_class_name] = dict(table)


def _module_of(hook: Callable):
    mod = getattr(hook, "__self__", None)
    if mod is None or getattr(hook, "__name__", "") != "execute":
        return None                    # get_detection_module_hooks registers module.execute
    return mod


def _spec(hook: Callable, hook_type: str, opcode: str):
    mod = _module_of(hook)
    if mod is None:
        return None
    table = BATCH_SAFE.get(type(mod).__name__)
    if table is None:
        return None
    return table.get((hook_type, opcode))


def _resolve_types(mod, names) -> Tuple[type, ...]:
    """Classes named `names` in the module's Python module -- or, for a name it
    does not import, in the modules its imported functions come from (the
    reference's state_change_external_calls.py imports
    get_potential_issues_annotation, not PotentialIssuesAnnotation)."""
    import sys
    pymod = sys.modules.get(type(mod).__module__)
    out = []
    for n in names:
        t = getattr(pymod, n, None)
        if not isinstance(t, type):
            for v in list(vars(pymod).values()) if pymod is not None else ():
                home = sys.modules.get(getattr(v, "__module__", None) or "")
                if callable(v) and home is not None and isinstance(getattr(home, n, None), type):
                    t = getattr(home, n)
                    break
        if isinstance(t, type):
            out.append(t)
    return tuple(out)


class TaintPlan:
    """What the device does for a LaserEVM's registered hooks.  `prev`: the plan
    this one replaces mid-batch; its replay tables stay (the device may already
    have applied its actions, and their records and sinks replay later)."""

    def __init__(self, laser, prev: Optional["TaintPlan"] = None):
        self.actions = np.zeros(256, dtype=np.uint32)
        self.safe: set = set()                         # opcode bytes the device no longer stops at
        self.pre_replay: Dict[int, List[Callable]] = {}
        self.post_replay: Dict[int, List[Callable]] = {}
        self.pre_operand: Dict[int, int] = {}
        self.sink: Optional[Tuple[Callable, str, int]] = None
        self.yield_types: Tuple[type, ...] = ()
        self.modules: List = []
        self.op_modules: Dict[int, List] = {}          # safe opcode -> modules hooked on it
        self.deferred: Dict[int, List[Callable]] = {}    # opcode -> Deferred hooks, in order
        self.iflane_types: Tuple[type, ...] = ()
        self.iflane_missing: Tuple[type, ...] = ()     # yield while the state lacks one
        if laser._execute_state_hooks:
            return                                     # every opcode is a host event anyway
        sink_mod = None
        for name, op in OPCODES.items():
            if laser.instr_pre_hook.get(name) or laser.instr_post_hook.get(name):
                continue
            pre, post = laser.pre_hooks.get(name, []), laser.post_hooks.get(name, [])
            if not pre and not post:
                continue
            specs_pre = [(h, _spec(h, "pre", name)) for h in pre]
            specs_post = [(h, _spec(h, "post", name)) for h in post]
            if any(s is None for _, s in specs_pre + specs_post):
                continue
            if any(not isinstance(s, AnnotateResult) for _, s in specs_post):
                continue
            ann = [s for _, s in specs_pre if isinstance(s, Annotate)]
            sinks = [(h, s) for h, s in specs_pre if isinstance(s, Sink)]
            yields = [(h, s) for h, s in specs_pre if isinstance(s, YieldIf)]
            defers = [(h, s) for h, s in specs_pre if isinstance(s, Deferred)]
            ifsyms = [s for _, s in specs_pre if isinstance(s, IfSymbolic)]
            iflanes = [(h, s) for h, s in specs_pre if isinstance(s, IfStateAnnotation)]
            if len({s.operand for s in ifsyms}) > 1 or any(s.operand > 6 for s in ifsyms):
                continue
            if any(not 1 <= s.words <= 3 for _, s in defers):
                continue
            if any(len(_resolve_types(_module_of(h), s.missing)) != len(s.missing) for h, s in iflanes):
                continue                                # a side effect the host cannot see: host hooks
            if len({a.operand for a in ann}) > 1 or any(a.operand > 1 for a in ann):
                continue
            if len({s.operand for _, s in sinks}) > 1 or len({s.operand for _, s in yields}) > 1:
                continue
            if sinks and sink_mod is not None and any(_module_of(h) is not sink_mod for h, _ in sinks):
                continue                                # one sink module per batch
            if any(s.operand > 6 for _, s in sinks + yields):
                continue
            word = 0
            if ann:
                word |= ann[0].operand + 1
                if any(a.exp_cond for a in ann):
                    if not all(a.exp_cond for a in ann):
                        continue
                    word |= MG_TAINT_EXPCOND
                if any(a.yield_class for a in ann):
                    word |= MG_TAINT_YCLASS
                self.pre_replay[op] = [h for h, s in specs_pre if isinstance(s, Annotate)]
                self.pre_operand[op] = ann[0].operand
            if specs_post:
                word |= MG_TAINT_POST
                if any(s.yield_class for _, s in specs_post):
                    word |= MG_TAINT_YCLASS
                self.post_replay[op] = [h for h, _ in specs_post]
            if sinks:
                word |= (sinks[0][1].operand + 1) << MG_TAINT_SINK_SHIFT
                sink_mod = _module_of(sinks[0][0])
                self.sink = (sinks[0][0], name, sinks[0][1].operand)
            if yields:
                word |= (yields[0][1].operand + 1) << MG_TAINT_YIELD_SHIFT
                for h, s in yields:
                    self.yield_types += _resolve_types(_module_of(h), s.types)
            if defers:
                word |= max(s.words for _, s in defers) << MG_TAINT_DEFER_SHIFT
                self.deferred[op] = [h for h, _ in defers]
            if ifsyms:
                word |= (ifsyms[0].operand + 1) << MG_TAINT_IFSYM_SHIFT
            if iflanes:
                word |= MG_TAINT_IFLANE
                for h, s in iflanes:
                    self.iflane_types += _resolve_types(_module_of(h), s.types)
                    self.iflane_missing += _resolve_types(_module_of(h), s.missing)
            self.actions[op] = word
            self.safe.add(op)
            mods = []
            for h, _ in specs_pre + specs_post:
                m = _module_of(h)
                if all(m is not x for x in mods):
                    mods.append(m)
                if all(m is not x for x in self.modules):
                    self.modules.append(m)
            self.op_modules[op] = mods
        if prev is not None:
            for k, v in prev.pre_replay.items():
                self.pre_replay.setdefault(k, v)
            for k, v in prev.post_replay.items():
                self.post_replay.setdefault(k, v)
            for k, v in prev.pre_operand.items():
                self.pre_operand.setdefault(k, v)
            if self.sink is None:
                self.sink = prev.sink
            for k, v in prev.deferred.items():
                self.deferred.setdefault(k, v)
            self.yield_types = tuple(dict.fromkeys(self.yield_types + prev.yield_types))
            for m in prev.modules:
                if all(m is not x for x in self.modules):
                    self.modules.append(m)

    @property
    def active(self) -> bool:
        return bool(self.safe)

    def key(self):
        """Changes when a module's issue cache does (the forced addresses change)."""
        return tuple(len(getattr(m, "cache", ()) or ()) for m in self.modules)

    def force_flags(self, code) -> np.ndarray:
        """Per instruction of `code` (mg_taint_force): DetectionModule.execute
        returns early at an address in the module's issue cache (base.py:79-86).
        2 = every module hooked on the opcode has the address cached: the device
        skips the actions; 1 = some of them have: the lane stops and the host runs
        the hooks.  The cache's code key is the module's own business, so this is
        keyed by address only -- a stop where no issue was cached for this code is
        merely a host event, and a skip only happens where every module's cache
        names the address (a code whose module hooks would have run there is the
        case the key cannot separate; modules cache per code hash, so a batch of
        one code is exact)."""
        cached = []
        for m in self.modules:
            if getattr(m, "auto_cache", True):
                cached.append((m, {entry[0] for entry in getattr(m, "cache", ()) or ()}))
        ins = code.instruction_list
        flags = np.zeros(len(ins), dtype=np.uint8)
        if not any(c for _, c in cached):
            return flags
        where = {id(m): c for m, c in cached}
        for k, x in enumerate(ins):
            op = OPCODES.get(x["opcode"])
            if op not in self.safe:
                continue
            mods = self.op_modules.get(op, ())
            hit = [m for m in mods if x["address"] in where.get(id(m), ())]
            if hit:
                flags[k] = 2 if len(hit) == len(mods) else 1
        return flags


class LaneTaint:
    """Host side of one taint lane: handle -> object, atom -> annotation set."""
    __slots__ = ("objs", "atoms", "msets", "fn_pack")

    def __init__(self):
        self.objs: Dict[int, Expression] = {}
        self.atoms: List[Optional[frozenset]] = []
        self.msets: Dict[int, frozenset] = {}     # mask -> union of its (final) atom sets
        self.fn_pack: Optional[str] = None        # active_function_name when the lane was packed


def state_needs_taint(state) -> bool:
    """Whether a state carries annotations a concrete lane would drop."""
    env = state.environment
    for w in (getattr(env, a) for a in _ENV_ATTRS):
        if isinstance(w, Expression) and w.annotations:
            return True
    return any(isinstance(x, Expression) and x.annotations for x in state.mstate.stack)


def pack(b, i: int, state, lt: LaneTaint, plan: Optional[TaintPlan]) -> bool:
    """Write state's object graph into lane i's taint planes.  False when it needs
    more than 64 atoms or the object table (the lane cannot carry it)."""
    lt.objs, lt.atoms, lt.msets = {}, [], {}
    lt.fn_pack = state.environment.active_function_name
    atom_of: Dict[int, int] = {}
    keep = []

    def mask(o) -> int:
        m = 0
        for a in o.annotations:
            k = atom_of.get(id(a))
            if k is None:
                k = atom_of[id(a)] = len(lt.atoms)
                lt.atoms.append(frozenset((a,)))
                keep.append(a)
            m |= 1 << k
        return m

    handle: Dict[int, int] = {}
    row = b.omask[i]
    env = state.environment
    for k, attr in enumerate(_ENV_ATTRS):
        o = getattr(env, attr)
        row[k + 1] = 0
        if isinstance(o, Expression):
            handle[id(o)] = k + 1
            lt.objs[k + 1] = o
            row[k + 1] = mask(o)
    row[MG_TAINT_CDSIZE] = 0
    cd = env.calldata
    if hasattr(cd, "calldatasize") and not isinstance(cd, (bytes, bytearray)):
        o = cd.calldatasize
        if isinstance(o, Expression):
            handle[id(o)] = MG_TAINT_CDSIZE
            lt.objs[MG_TAINT_CDSIZE] = o
            row[MG_TAINT_CDSIZE] = mask(o)
    stack = state.mstate.stack
    counts = Counter(id(x) for x in stack)
    nxt = MG_TAINT_OBJ0
    cap = b.shape.obj_cap
    so = b.sobj[i]
    so[:] = 0
    for slot, x in enumerate(stack):
        h = handle.get(id(x))
        if h is None:
            if isinstance(x, Expression) and (counts[id(x)] > 1 or x.annotations):
                if nxt + 4 > cap:
                    return False
                h = handle[id(x)] = nxt
                nxt += 1
                lt.objs[h] = x
                row[h] = mask(x)
            else:
                h = 0
        so[slot] = h
    if len(lt.atoms) > MAX_ATOMS:
        return False
    b.n_obj[i] = b.n_fixed[i] = nxt
    b.n_atoms[i] = len(lt.atoms)
    b.sink[i] = 0
    b.tflags[i] = 0
    ym = 0
    if plan is not None and plan.yield_types:
        for k, s in enumerate(lt.atoms):
            if any(isinstance(a, plan.yield_types) for a in s):
                ym |= 1 << k
    b.ymask[i] = ym
    if plan is not None and ((plan.iflane_types and any(isinstance(a, plan.iflane_types)
                                                        for a in state.annotations))
                             or any(not any(isinstance(a, t) for a in state.annotations)
                                    for t in plan.iflane_missing)):
        b.tflags[i] = 2                    # MG_TAINT_IFLANE hooks have work on this path
    return True


def _bits(m: int):
    k = 0
    while m:
        if m & 1:
            yield k
        m >>= 1
        k += 1


def _world_view(ws, n_constraints: int):
    """The world state a replayed hook sees: the lane's (accounts, transaction
    sequence and annotations shared -- the batch-safe hooks only read them) with
    the path constraints it had at the hooked step."""
    view = object.__new__(type(ws))
    view.__dict__.update(ws.__dict__)
    view.constraints = list(ws.constraints[:n_constraints])
    return view


def _environment_at(state, fent: int, fn_pack: Optional[str]):
    """The lane's environment as the hook saw it: a copy carrying the function
    name of that step -- the record's last function-entry landing
    (mg_lane_soa.fent, svm.py:575-637), or the name the lane was packed with
    when it had not landed on one yet.  A copy: the reference steps copies,
    so a state a hook keeps (an OverUnderflowAnnotation's overflowing_state)
    keeps the name it had."""
    from copy import copy
    from .transaction import ContractCreationTransaction
    env = copy(state.environment)
    seq = state.world_state.transaction_sequence
    if fent == 0xFFFFFFFF:
        if fn_pack is not None:
            env.active_function_name = fn_pack
    elif seq and isinstance(seq[-1], ContractCreationTransaction):
        env.active_function_name = "constructor"
    else:
        name = env.code.name_at(fent)
        if name is not None:
            env.active_function_name = name
    return env


def _snapshot(state, pc: int, stack, n_constraints: int, env=None):
    """The state a replayed hook sees: the lane's environment (as of the step,
    `env`) and transaction, the world state with the path constraints the lane
    had at that step, pc and the recorded stack words.  Memory and storage are
    not reproduced (the batch-safe hooks do not read them)."""
    from .state import GlobalState, MachineState
    ws = _world_view(state.world_state, n_constraints)
    ms = MachineState(gas_limit=state.mstate.gas_limit, pc=pc, stack=stack, depth=state.mstate.depth)
    g = GlobalState(ws, state.environment if env is None else env, state.node, ms,
                    transaction_stack=list(state.transaction_stack), last_return_data=state.last_return_data)
    return g


def note_record(lt: LaneTaint, rec, state, plan: TaintPlan) -> None:
    """An MG_REC_ANNOT record, replayed in the reference's global execution order
    (LaserEVM._replay_records): the module's own hook runs now, on a state built
    from the record, so it sees the module's caches and the path's constraints
    as they are at that step; what it annotates becomes the atom's set."""
    _step, _kind, atom, pc, op, post, v0, v1, fent = rec
    while len(lt.atoms) <= atom:
        lt.atoms.append(None)
    o0, o1 = symbol_factory.BitVecVal(v0, 256), symbol_factory.BitVecVal(v1, 256)
    if post:
        target = o0
        hooks = plan.post_replay.get(op, ())
        pc_at = pc + 1                     # the post-hook state is the successor
    else:
        target = o0 if plan.pre_operand.get(op, 0) == 0 else o1
        hooks = plan.pre_replay.get(op, ())
        pc_at = pc
    snap = _snapshot(state, pc_at, [o1, o0], len(state.world_state.constraints),
                     _environment_at(state, fent, lt.fn_pack))
    for h in hooks:
        h(snap)
    lt.atoms[atom] = frozenset(target.annotations)


def replay_deferred(rec, state, plan: TaintPlan, lt: Optional[LaneTaint] = None) -> None:
    """An MG_REC_HOOK record, in the reference's global execution order: the
    opcode's deferred hooks (the modules' own `execute`) run on a state with the
    recorded words, pc and path constraints as of that step, sharing the lane's
    state and world-state annotations, so what they file lands where the
    reference's hooks put it."""
    from .state import GlobalState, MachineState
    _step, _kind, words, pc, op, fent = rec
    ws = _world_view(state.world_state, len(state.world_state.constraints))
    stack = [symbol_factory.BitVecVal(w, 256) for w in reversed(words)]
    env = _environment_at(state, fent, lt.fn_pack if lt is not None else None)
    snap = GlobalState(ws, env, state.node,
                       MachineState(gas_limit=state.mstate.gas_limit, pc=pc, stack=stack,
                                    depth=state.mstate.depth),
                       transaction_stack=list(state.transaction_stack), last_return_data=state.last_return_data)
    snap._annotations = state._annotations
    for h in plan.deferred.get(op, ()):
        h(snap)


def atoms_set(lt: LaneTaint, m: int) -> frozenset:
    """The annotation set of mask `m` (every atom was resolved when its record
    was replayed, or at pack).  An atom's set never changes once resolved, so
    the union is memoised per mask until the next pack renumbers the atoms."""
    m = int(m)
    got = lt.msets.get(m)
    if got is not None:
        return got
    out = frozenset()
    for k in _bits(m):
        got = lt.atoms[k] if k < len(lt.atoms) else None
        if got is None:
            raise RuntimeError(f"taint atom {k} has no record")
        out = out | got
    lt.msets[m] = out
    return out


def materialise(b, i: int, state, lt: LaneTaint, plan: TaintPlan, words: list) -> list:
    """Lane i's stack as objects: `words` are fresh objects for its values; slots
    that share a handle become one object, handles the host packed become the
    very objects it packed, each with the annotation set of its mask.  The
    environment words' sets are updated in place and the sink hook, when one
    ran, is replayed on `state`.  Every handle is fixed afterwards."""
    row = b.omask[i]
    so = b.sobj[i]
    made: Dict[int, Expression] = {}
    seen = set()
    out = []
    for slot, x in enumerate(words):
        h = int(so[slot])
        if h == 0:
            if x.annotations or id(x) in seen:
                x = type(x)(x.raw)          # an object of its own, as the reference's push made it
            seen.add(id(x))
            out.append(x)
            continue
        o = made.get(h)
        if o is None:
            ann = atoms_set(lt, int(row[h]))
            o = lt.objs.get(h)
            if o is None:
                o = type(x)(x.raw, ann)
                lt.objs[h] = o
            elif not ann <= o.annotations:
                o.annotations = o.annotations | ann
            made[h] = o
        out.append(o)
    for h in range(1, MG_TAINT_CDSIZE + 1):
        o = lt.objs.get(h)
        if o is not None and int(row[h]):
            ann = atoms_set(lt, int(row[h]))
            if not ann <= o.annotations:
                o.annotations = o.annotations | ann
    if int(b.tflags[i]) & 1 and plan.sink is not None:
        replay_sink(state, atoms_set(lt, int(b.sink[i])), plan)
        b.tflags[i] = 0
        b.sink[i] = 0
    b.n_fixed[i] = b.n_obj[i]
    return out


def replay_sink(state, ann: frozenset, plan: TaintPlan) -> None:
    """Run the sink module's own hook once on `state` (sharing its annotation
    list) with stack[-1-operand] carrying `ann`: the module adds them to its
    state annotation exactly as its SSTORE/JUMPI pre-hooks would have."""
    from .state import GlobalState, MachineState
    hook, opname, operand = plan.sink
    instrs = state.environment.code.instruction_list
    pc = next((k for k, ins in enumerate(instrs) if ins["opcode"] == opname), None)
    if pc is None:
        return
    word = symbol_factory.BitVecVal(0, 256, ann)
    stack = [word] + [symbol_factory.BitVecVal(0, 256) for _ in range(operand)]
    proxy = GlobalState(state.world_state, state.environment, state.node,
                        MachineState(gas_limit=state.mstate.gas_limit, pc=pc, stack=stack),
                        transaction_stack=state.transaction_stack, last_return_data=state.last_return_data)
    proxy._annotations = state._annotations
    hook(proxy)
