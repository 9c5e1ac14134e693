"""Feasibility checks with kernel 2 as the quick-sat prefilter.

Mirrors, with the same names, arguments and error behaviour:

* ``LRUCache`` / ``ModelCache`` (support/support_utils.py:34-68): the 100 most
  recently used models; ``check_quick_sat(expr)`` returns the first model in
  most-recently-used order under which the expression is true, moves it to
  most-recent, and memoises per expression (``lru_cache(2**10)``).  The models
  are evaluated on kernel 2 (``mg_eval``), all of them in one launch;
  ``check_quick_sat_many`` evaluates a whole sequence of queries in one launch
  (``mg_eval_bits``) and replays the sequential calls exactly, LRU moves
  included.
* ``get_model`` (support/model.py:21-82): ``lru_cache(2**23)``; a literal False
  raises UnsatError; quick-sat only when nothing is minimised or maximised;
  otherwise the SMT backend, whose model is cached with count 1.
* ``Constraints`` (state/constraints.py:12-131): ``is_possible`` maps a timeout to
  False (default timeout) or True (custom timeout) and UnsatError to False;
  ``get_all_constraints`` appends the keccak conjunct.

The prefilter only ever answers SAT with a model.  A constraint set the device
cannot evaluate (flatten.Unsupported) and a set no cached model satisfies both
fall through to the backend unchanged.  The backend is z3 in the reference; z3
is not installed in this image nor on the GPU box, so ``solver_backend`` is a
pluggable callable (constraints, minimize, maximize, timeout_ms) -> model that
raises UnsatError / SolverTimeOutException.  Without one installed, a
quick-sat miss raises SolverBackendMissing: it is never mapped to "unsat" or
"timeout", so no feasible path is ever pruned silently.
"""
from __future__ import annotations

import os
import time
from collections import OrderedDict
from functools import lru_cache
from typing import Callable, Dict, Iterable, List, Optional, Sequence

import numpy as np

from .expr import And, BitVec, Bool, Node, TRUE, _fold, _select, const, symbol_factory
from .flatten import Compiler, batch_from, compile_sets
from .lower import Unsupported
from .program import ArrayInterp, FuncInterp, ModelPool, PoolColumns, compact_vars, concat_pools, read_sets

NO_MODEL = 0xFFFFFFFF


class UnsatError(Exception):
    """mythril/exceptions.py: the constraints are unsatisfiable."""


class SolverTimeOutException(UnsatError):
    """mythril/exceptions.py:23: the solver gave up -- an UnsatError, as there:
    a module that catches UnsatError treats a timeout as "no issue"."""


class SolverBackendMissing(RuntimeError):
    """Kernel 2 found no cached model and no SMT backend is installed, so the
    query cannot be decided.  Deliberately not a SolverTimeOutException /
    UnsatError: is_possible() would turn either into a silent prune."""


def simplify(expr):
    """Expressions are folded as they are built (expr._fold, lower._select), so
    simplify returns its argument."""
    return expr


# ------------------------------------------------------------------ models
def _decl(node: Node):
    """Name of the declaration an expression applies (z3 ``expr.decl()``) when a
    model can declare it: a variable, an uninterpreted function or an array."""
    if node.op in ("var", "array"):
        return node.param if node.op == "var" else node.param[0]
    if node.op == "uf":
        return node.param[0]
    return None


class ModelRef:
    """One interpretation (z3.ModelRef): variable values by name (Bools 0/1),
    ArrayInterp per symbolic array, FuncInterp per uninterpreted function.
    Hashed by identity, as z3 models are."""

    def __init__(self, assignment: Optional[Dict[str, object]] = None):
        self.assignment: Dict[str, object] = dict(assignment or {})

    def decls(self) -> List[str]:
        return list(self.assignment)

    def __getitem__(self, name):
        return self.assignment.get(name)

    def get(self, name: str, default=None):
        return self.assignment.get(name, default)

    def eval(self, expression, model_completion: bool = False):
        """z3 ModelRef.eval: substitute the interpretation and simplify (the
        builders fold constant operands, expr._fold).  Without completion,
        declarations the model lacks stay symbolic; with it they take 0 (BV),
        False (Bool), a 0 array default, a 0 function else-value."""
        raw = expression.raw if hasattr(expression, "raw") else expression
        out = _substitute(raw, self.assignment, model_completion, {})
        if isinstance(expression, Bool):
            return Bool(out)
        if isinstance(expression, BitVec):
            return BitVec(out)
        return out

    def __repr__(self):
        return f"ModelRef({self.assignment})"


def _substitute(node: Node, asg, completion: bool, memo) -> Node:
    got = memo.get(id(node))
    if got is not None:
        return got
    op = node.op
    if op in ("const", "array"):
        out = node
    elif op == "var":
        v = asg.get(node.param)
        if v is None and completion:
            v = 0
        out = node if v is None else const(int(v), node.width)
    else:
        args = tuple(_substitute(a, asg, completion, memo) for a in node.args)
        if op == "select":
            out = _select(args[0], args[1])
            if out.op == "select" and out.args[0].op == "array" and out.args[1].op == "const":
                interp = asg.get(out.args[0].param[0])
                if isinstance(interp, ArrayInterp):
                    out = const(interp.entries.get(out.args[1].param, interp.default), out.width)
                elif completion:
                    out = const(0, out.width)
        elif op == "uf":
            out = Node(op, node.width, args, node.param)
            if all(a.op == "const" for a in args):
                interp = asg.get(node.param[0])
                if isinstance(interp, FuncInterp):
                    key = tuple(a.param for a in args)
                    out = const(interp.entries.get(key, interp.else_value), node.width)
                elif completion:
                    out = const(0, node.width)
        elif op in ("store", "K"):
            out = Node(op, node.width, args, node.param)
        else:
            out = _fold(op, node.width, args, node.param)
    memo[id(node)] = out
    return out


class Model:
    """laser/smt/model.py:6-59: a model made of several internal models (the
    independence solver's per-bucket models).  ``eval`` uses the first internal
    model that declares the expression's declaration, else the last one;
    ``__getitem__`` the first that interprets the item.  ``Model(dict)`` is
    shorthand for one internal model with that assignment."""

    def __init__(self, models=None):
        if isinstance(models, dict):
            models = [ModelRef(models)]
        elif isinstance(models, ModelRef):
            models = [models]
        self.raw: List[ModelRef] = list(models or [])

    def decls(self) -> List[str]:
        out: List[str] = []
        for m in self.raw:
            out.extend(m.decls())
        return out

    def __getitem__(self, item):
        if isinstance(item, int):
            return self.decls()[item]
        for m in self.raw:
            r = m[item]
            if r is not None:
                return r
        return None

    def get(self, name: str, default=None):
        r = self[name]
        return default if r is None else r

    def view(self, expression) -> Optional[ModelRef]:
        """The internal model ``eval(expression)`` uses."""
        raw = expression.raw if hasattr(expression, "raw") else expression
        d = _decl(raw)
        for k, m in enumerate(self.raw):
            if (d is not None and d in m.assignment) or k == len(self.raw) - 1:
                return m
        return None

    def eval(self, expression, model_completion: bool = False):
        m = self.view(expression)
        return None if m is None else m.eval(expression, model_completion)

    @property
    def assignment(self) -> Dict[str, object]:
        """The interpretation quick-sat evaluates a conjunction under: And has no
        declaration a model can declare, so the last internal model."""
        return self.raw[-1].assignment if self.raw else {}

    def __repr__(self):
        return f"Model({[m.assignment for m in self.raw]})"


class LRUCache:
    def __init__(self, size):
        self.size = size
        self.lru_cache: "OrderedDict" = OrderedDict()

    def get(self, key):
        try:
            value = self.lru_cache.pop(key)
            self.lru_cache[key] = value
            return value
        except KeyError:
            return -1

    def put(self, key, value):
        try:
            self.lru_cache.pop(key)
        except KeyError:
            if len(self.lru_cache) >= self.size:
                self.lru_cache.popitem(last=False)
        self.lru_cache[key] = value


_MISSING = object()


class _RowGen:
    """Conjunct rows (bool per model, in the generation's first pool order) of
    one pool generation (ModelCache._row_gen)."""

    def __init__(self, head: List, seeds: List):
        # the generation keeps its models (and the seed list) alive: no model
        # made later can take one's id while the rows exist
        self.head, self.seeds = head, seeds
        self.head_ids = [id(m) for m in head]
        self.head_pos = {i: k for k, i in enumerate(self.head_ids)}
        self.rows: Dict[Node, np.ndarray] = {}


def _fingerprint(m) -> tuple:
    """A head model's identity and its interpretations' identity and size (an
    interpretation replaced or extended makes another generation)."""
    if isinstance(m, Model):
        return (id(m),) + tuple((id(r.assignment), len(r.assignment)) for r in m.raw)
    return (id(m),)


def _pack_bits(b: np.ndarray) -> np.ndarray:
    """bool per model -> the uint64 bitmap words eval_bits returns."""
    words = (len(b) + 63) // 64
    out = np.zeros(words * 8, dtype=np.uint8)
    packed = np.packbits(b, bitorder="little")
    out[:len(packed)] = packed
    return out.view(np.uint64)


def _valid_bits(n: int) -> np.ndarray:
    """The bitmap (uint64 words, bit i of word i >> 6) with the first n bits set."""
    valid = np.zeros((n + 63) // 64, dtype=np.uint64)
    full, rest = divmod(n, 64)
    valid[:full] = np.uint64(0xFFFFFFFFFFFFFFFF)
    if rest:
        valid[full] = np.uint64((1 << rest) - 1)
    return valid


def _raw(expr) -> Node:
    return expr.raw if isinstance(expr, Bool) else expr


class ModelCache:
    QUICK_SAT_MEMO = 2 ** 10

    def __init__(self, device=None):
        self.model_cache = LRUCache(size=100)
        self._device = device
        self._memo: "OrderedDict[Node, object]" = OrderedDict()
        self._fresh: List = []          # models this rank found since the last exchange
        self.device_evals = 0          # constraint-evals run on kernel 2
        self.launches = 0
        self.device_ms = 0.0           # kernel-2 time of those launches
        # candidate models beyond the LRU (witness seeds, SURVEY §8(b): kernel 2
        # evaluates thousands where the reference keeps 100): consulted only
        # where the reference would call its SMT backend, see get_model
        self.seeds: List = []
        self._seed_list = None
        # an object with models() and epoch (laser/witness.WitnessSeeds), or None
        self.seed_source = None
        self._seed_cols = None               # (epoch, PoolColumns) of the seeds
        # quick-sat bitmaps computed ahead for a group of queries (prefetch)
        self._bits: Dict[Node, tuple] = {}
        self._seed_memo: Dict[Node, object] = {}
        self._compiler = None                 # persistent: conjunct programs are compiled once
        self._progs: Dict[Node, object] = {}
        self.part_evals = 0            # conjunct programs x models run on kernel 2
        self._rowgens: "OrderedDict[tuple, _RowGen]" = OrderedDict()
        # conjunct rows by model (_rows_by_model): the seed block per seed epoch,
        # head models' bits by fingerprint (models kept alive in _head_keep)
        self._seed_sig = None
        self._seed_rows: Dict[Node, np.ndarray] = {}
        self._head_bits: Dict[Node, Dict[tuple, bool]] = {}
        self._head_keep: Dict[tuple, object] = {}
        self.stats = {"queries": 0, "lru_hits": 0, "seed_hits": 0, "misses": 0, "divergences": 0}

    @property
    def device(self):
        if self._device is None:
            from ..device import GpuDevice
            self._device = GpuDevice(int(os.environ.get("LOCAL_RANK", "0")))
        return self._device

    def put(self, key, value, peer: bool = False):
        """Cache a model (support_utils.py:34-53 put).  peer=True: a model another
        rank found (§8(e) all-gather), not re-shared at the next exchange."""
        self.model_cache.put(key, value)
        if not peer:
            self._fresh.append(key)
            if len(self._fresh) > self.model_cache.size:     # older ones are evicted anyway
                del self._fresh[0]

    def take_fresh(self) -> List:
        """Models this rank cached since the last call (for the all-gather)."""
        out, self._fresh = self._fresh, []
        return out

    # -- memo = functools.lru_cache(maxsize=2**10) on check_quick_sat ---------
    def _memo_get(self, key):
        if key in self._memo:
            self._memo.move_to_end(key)
            return True, self._memo[key]
        return False, None

    def _memo_put(self, key, value):
        self._memo[key] = value
        self._memo.move_to_end(key)
        if len(self._memo) > self.QUICK_SAT_MEMO:
            self._memo.popitem(last=False)

    def _seed_tailed(self, models: List) -> bool:
        """Whether _pool takes the seed block from cached columns (the models end
        with the seed list)."""
        seeds = self.seeds
        n = len(models) - len(seeds)
        return bool(seeds) and n >= 0 and all(a is b for a, b in zip(models[n:], seeds))

    def _pool(self, models: List[Model], prog, key: Optional[Node] = None) -> ModelPool:
        seeds = self.seeds
        n = len(models) - len(seeds)
        if seeds and n >= 0 and all(a is b for a, b in zip(models[n:], seeds)):
            # the seed block comes from cached columns (rebuilt when the seeds change)
            if self._seed_cols is None or self._seed_cols[0] is not self.seed_source or \
                    len(self._seed_cols[1].assigns) != len(seeds):
                cols = PoolColumns([_view(m, None) for m in seeds],
                                   getattr(self.seed_source, "revision", None))
                self._seed_cols = (self.seed_source, cols)
            block = self._seed_cols[1].pool(prog.var_names, prog.var_widths, prog.tables)
            if n == 0:
                return block
            # the head's models over the variables these programs read only (the
            # batch keeps the compiler's numbering for the seed block's columns)
            head = ModelPool.from_dicts([_view(m, key) for m in models[:n]], prog.var_names,
                                        prog.var_widths, prog.tables, reads=read_sets(prog))
            return concat_pools(head, block)
        return ModelPool.from_dicts([_view(m, key) for m in models], prog.var_names,
                                    prog.var_widths, prog.tables)

    def _select(self, model: Model) -> Model:
        self.model_cache.put(model, self.model_cache.get(model) + 1)
        return model

    def check_quick_sat(self, constraints):
        key = _raw(constraints)
        hit, val = self._memo_get(key)
        if hit:
            return val
        result = False
        if self.seed_source is not None:
            self._seed_models()          # seeds in the LRU are completed for every input first
        models = list(reversed(self.model_cache.lru_cache.keys()))      # MRU first
        if models:
            pre = self._bits.get(key)
            if pre is None or not all(id(m) in pre[0] for m in models):
                pre = self._eval_keys([key], self._full_pool(models), keep=False).get(key)
            if pre is not None:
                pos, row = pre[0], pre[1]
                for m in models:
                    p = pos[id(m)]
                    if (int(row[p >> 6]) >> (p & 63)) & 1:
                        result = self._select(m)
                        break
        self._memo_put(key, result)
        return result

    # -- evaluation by conjuncts ----------------------------------------------------
    def _eval_keys(self, keys: Sequence[Node], pool: List, keep: bool = True) -> Dict[Node, tuple]:
        """Per key, (position of each pool model, satisfied-model bitmap), from ONE
        kernel-2 launch.  A key is a conjunction (get_model's And of the path
        constraints and the keccak conjunct): it is taken apart into its
        conjuncts, each distinct conjunct of the whole group is compiled and
        evaluated once, and a key's bitmap is the AND of its conjuncts' -- the
        same truth as the conjunction evaluated whole, for a fraction of the
        compile work (sibling paths share most conjuncts, and every query of a
        group shares the keccak conjunct).  Keys with a conjunct the device does
        not evaluate get no entry (they stay with the backend)."""
        out: Dict[Node, tuple] = {}
        if not pool or not keys:
            return out
        if any(_decl(k) is not None for k in keys) and any(isinstance(m, Model) and len(m.raw) > 1 for m in pool):
            return out                        # a per-query internal model: evaluate on the host path
        parts_of = {}
        distinct: "OrderedDict[Node, None]" = OrderedDict()
        for k in keys:
            cs = _conjuncts(k)
            parts_of[k] = cs
            for c in cs:
                distinct[c] = None
        plist = [c for c in distinct if c.op != "const"]
        rows = self.conjunct_rows(plist, pool)
        ones = _valid_bits(len(pool))
        # a model's first position (the dict keeps the last write: build back to front)
        n = len(pool)
        pos = dict(zip(map(id, reversed(pool)), range(n - 1, -1, -1)))
        # the bitmaps place models by id(): the entry keeps its pool's models
        # alive, so no model created later (after an LRU eviction frees one)
        # can take a dead model's id and read its bit
        alive = tuple(pool)
        # the seeds as a contiguous tail of the pool (its usual shape, _full_pool):
        # check_seeds then reads the first satisfying seed off the bitmap
        ns = len(self.seeds)
        tail = (self.seeds, len(pool) - ns) if ns and len(pool) >= ns and \
            all(a is b for a, b in zip(pool[len(pool) - ns:], self.seeds)) else None
        for k in keys:
            acc = ones.copy()
            ok = True
            for c in parts_of[k]:
                if c.op == "const":
                    if not c.param:
                        acc[:] = 0
                    continue
                r = rows.get(c)
                if r is None:
                    ok = False
                    break
                acc &= r
            if ok:
                out[k] = (pos, acc, alive, tail)
                self.device_evals += len(pool)
        if keep:
            self._bits.update(out)
        return out

    def conjunct_rows(self, conjuncts: Sequence[Node], pool: List, columns=None) -> Dict[Node, np.ndarray]:
        """Per conjunct, the bitmap of the pool's models that satisfy it, from
        ONE kernel-2 launch; conjuncts the device does not evaluate get no row.
        Every conjunct is compiled once per cache, by one compiler whose index
        spaces only grow (flatten.batch_from).

        A conjunct's truth under a model does not change while the model does
        not, so rows are kept per pool generation (_RowGen: the same head models
        and the same completed seeds, in any order) and only conjuncts new to the
        generation go to the device.  A path's constraints are its parent's plus
        one, so most of a fork group's conjuncts were evaluated by earlier groups
        (exceptions.sol.o -t 2: 89 % of them, over 3 generations in 150 groups)."""
        if not conjuncts or not pool:
            return {}
        if columns is not None:
            # a caller's own pool with its cached columns (program.PoolColumns over
            # the pool's assignments, in order): the search's starting pool
            return self._rows_uncached(conjuncts, pool, columns)
        split = self._seed_split(pool)
        if split is None:
            return self._rows_uncached(conjuncts, pool)
        return self._rows_by_model(conjuncts, pool, split)

    HEAD_BITS_MODELS = 4096

    def _seed_split(self, pool: List) -> Optional[int]:
        """The head length of a model-cache pool -- LRU models that are not
        seeds, then every seed (_full_pool) -- or None for any other pool (the
        search's candidates)."""
        seeds = self.seeds
        ns, n = len(seeds), len(pool)
        if not ns or n < ns or self.seed_source is None:
            return None
        h = n - ns
        if pool[h] is not seeds[0] or not all(a is b for a, b in zip(pool[h:], seeds)):
            return None
        return h

    def _rows_by_model(self, conjuncts: Sequence[Node], pool: List, h: int) -> Dict[Node, np.ndarray]:
        """Rows kept per conjunct and per model: the seed block's bits per seed
        epoch, each head model's bit by its fingerprint (identity and
        interpretation sizes).  A model that enters the LRU (every answer of the
        exact procedure puts one there) then costs one small launch over the new
        models alone, not the whole pool again for every conjunct a generation
        had already evaluated."""
        seeds = self.seeds
        n = len(pool)
        head = pool[:h]
        sig = (id(seeds), len(seeds), getattr(self.seed_source, "epoch", None))
        if self._seed_sig != sig:
            self._seed_sig, self._seed_rows = sig, {}
        if len(self._head_keep) > self.HEAD_BITS_MODELS:
            self._head_keep, self._head_bits = {}, {}
        fps = [_fingerprint(m) for m in head]
        for fp, m in zip(fps, head):
            self._head_keep.setdefault(fp, m)         # ids stay unique while a bit is kept
        srows, hbits = self._seed_rows, self._head_bits
        todo = [c for c in conjuncts if c not in srows and self._progs.get(c, _MISSING) is not None]
        if todo:
            # the seed block alone (its cached columns as they are, no head block
            # copied in front); the head models' bits follow below, over the
            # variables the programs read
            ns = n - h
            fresh = self._rows_uncached(todo, pool[h:])
            for c, r in fresh.items():
                srows[c] = np.unpackbits(r.view(np.uint8), bitorder="little")[:ns].astype(bool)
        # head models a kept conjunct has no bit for: one launch over them alone
        missing: "OrderedDict[tuple, object]" = OrderedDict()
        need = []
        for c in conjuncts:
            if c not in srows:
                continue
            hb = hbits.setdefault(c, {})
            lack = [k for k, fp in enumerate(fps) if fp not in hb]
            if lack:
                need.append(c)
                for k in lack:
                    missing.setdefault(fps[k], head[k])
        if need:
            sub = list(missing.values())
            sub_fps = list(missing.keys())
            fresh = self._rows_uncached(need, sub)
            for c, r in fresh.items():
                u = np.unpackbits(r.view(np.uint8), bitorder="little")[:len(sub)].astype(bool)
                hb = hbits[c]
                for fp, bit in zip(sub_fps, u):
                    hb.setdefault(fp, bool(bit))
        rows: Dict[Node, np.ndarray] = {}
        for c in conjuncts:
            sr = srows.get(c)
            if sr is None:
                continue
            hb = hbits[c]
            if any(fp not in hb for fp in fps):
                continue                              # not evaluable on these models
            u = np.empty(n, dtype=bool)
            u[:h] = [hb[fp] for fp in fps]
            u[h:] = sr
            rows[c] = _pack_bits(u)
        return rows

    ROW_GENERATIONS = 4

    def _row_gen(self, pool: List):
        """(generation, permutation) of a model-cache pool -- LRU models that are
        not seeds, then every seed (_full_pool) -- or None for any other pool (the
        search's candidates).  The permutation maps the pool's positions to the
        generation's first order (None when equal).  A generation is the head
        models, each with its interpretations' identity and size, and the seed
        list at one completion epoch (WitnessSeeds.models: completion changes the
        seeds in place, and only with the epoch)."""
        seeds = self.seeds
        ns, n = len(seeds), len(pool)
        if not ns or n < ns or self.seed_source is None:
            return None
        h = n - ns
        if pool[h] is not seeds[0] or not all(a is b for a, b in zip(pool[h:], seeds)):
            return None
        head = pool[:h]
        fps = frozenset(_fingerprint(m) for m in head)
        if len(fps) != h:
            return None
        sig = (fps, id(seeds), ns, getattr(self.seed_source, "epoch", None))
        gens = self._rowgens
        gen = gens.get(sig)
        if gen is None:
            if len(gens) >= self.ROW_GENERATIONS:
                del gens[next(iter(gens))]
            gen = gens[sig] = _RowGen(head, seeds)
        ids = [id(m) for m in head]
        if ids == gen.head_ids:
            return gen, None
        perm = np.arange(n)
        perm[:h] = [gen.head_pos[i] for i in ids]
        return gen, perm

    def _rows_uncached(self, conjuncts: Sequence[Node], pool: List, columns=None) -> Dict[Node, np.ndarray]:
        rows: Dict[Node, np.ndarray] = {}
        if self._compiler is None:
            self._compiler = Compiler()
        progs, kept = [], []
        # a fork's two successors add X and its negation: the negation's bitmap is
        # the complement of X's over the pool (both are evaluated exactly, per
        # model), so only one of the pair is compiled and evaluated
        derived: Dict[Node, Node] = {}
        want = OrderedDict.fromkeys(conjuncts)
        for c in conjuncts:
            if c in derived:
                continue
            q = _complement(c)
            if q is not None and q in want and q not in derived and self._progs.get(c, _MISSING) is _MISSING \
                    and self._progs.get(q, _MISSING) is not None:
                derived[c] = q
        for c in [c for c in conjuncts if c not in derived] + [q for q in derived.values() if q not in want]:
            pr = self._progs.get(c, _MISSING)
            if pr is _MISSING:
                try:
                    pr = self._compiler.compile(c)
                except Unsupported:
                    pr = None
                self._progs[c] = pr
            if pr is not None:
                progs.append(pr)
                kept.append(c)
        if kept:
            prog = batch_from(self._compiler, progs)
            if columns is not None:
                mp = columns.pool(prog.var_names, prog.var_widths, prog.tables)
            else:
                if not self._seed_tailed(pool):
                    # a pool built from model dicts: only the variables and tables
                    # these programs read (the seed block keeps the compiler's
                    # numbering: its columns are cached by it)
                    prog = compact_vars(prog)
                mp = self._pool(pool, prog)
            _, _, bits, ms = self.device.eval_bits(prog, mp)
            self.part_evals += len(kept) * len(pool)
            self.device_ms += float(ms or 0.0)
            self.launches += 1
            for row, c in enumerate(kept):
                rows[c] = bits[row]
        if derived:
            valid = _valid_bits(len(pool))
            for c, q in derived.items():
                r = rows.get(q)
                if r is not None:
                    rows[c] = ~r & valid
        return rows

    # -- witness seeds and prefetched groups ------------------------------------
    def _seed_models(self) -> List:
        if self.seed_source is not None:
            ms = self.seed_source.models()
            # a seed source keeps its Model objects (completion updates them in
            # place): the list is re-taken only when the source hands out another
            if ms is not self._seed_list or len(ms) != len(self.seeds):
                self._seed_list = ms
                self.seeds = list(ms)
        return self.seeds

    def prefetch(self, raws: Sequence[Node]) -> None:
        """Quick-sat bitmaps of a group of queries (the fork filters of one BFS
        round, a transaction's reachability filter) against the current LRU
        models and the seeds, in ONE kernel-2 launch; check_quick_sat /
        check_seeds then replay the sequential reference order from them (LRU
        moves exactly as query by query)."""
        self._seed_models()
        pool = self._full_pool(list(reversed(self.model_cache.lru_cache.keys())))
        fresh = list(OrderedDict.fromkeys(
            k for k in raws if k not in self._bits and not (k in self._memo and k in self._seed_memo)))
        self._eval_keys(fresh, pool)

    def _full_pool(self, lru: List) -> List:
        """The LRU's models that are not seeds, then every seed (a pool's order
        only places bits: answers follow the LRU's MRU order, then the seeds')."""
        if not self.seeds:
            return lru
        ids = {id(m) for m in self.seeds}
        return [m for m in lru if id(m) not in ids] + self.seeds

    def clear_prefetch(self) -> None:
        self._bits.clear()

    def check_seeds(self, key: Node):
        """The first seed model (pool order) satisfying `key`, or None: where
        the reference asks its SMT backend for a model, a seed that satisfies
        the query is such a model (sound: it is checked, not guessed).  The
        answer is memoised: seeds only gain interpretations of inputs a query
        registered later, which it does not mention."""
        if key in self._seed_memo:
            return self._seed_memo[key]
        seeds = self._seed_models()
        if not seeds:
            return None
        pre = self._bits.get(key)
        if pre is None or pre[3] is None or pre[3][0] is not seeds:
            pre = self._eval_keys([key], seeds, keep=False).get(key)
        found = None
        if pre is not None and pre[3] is not None:
            off = pre[3][1]
            hit = np.unpackbits(pre[1].view(np.uint8), bitorder="little")[off:off + len(seeds)]
            if hit.any():
                found = seeds[int(np.argmax(hit))]
        self._seed_memo[key] = found
        return found

    def check_quick_sat_many(self, queries: Sequence) -> List[object]:
        """[check_quick_sat(q) for q in queries], with every query not already
        memoised evaluated against the current pool in ONE kernel-2 launch."""
        keys = [_raw(q) for q in queries]
        models0 = list(reversed(self.model_cache.lru_cache.keys()))
        pos0 = {id(m): i for i, m in enumerate(models0)}
        fresh = list(OrderedDict.fromkeys(k for k in keys if k not in self._memo))
        if any(_decl(k) is not None for k in fresh) and \
                any(isinstance(m, Model) and len(m.raw) > 1 for m in models0):
            # a bare declaration picks a per-query internal model: sequential path
            return [self.check_quick_sat(k) for k in keys]
        bits: Dict[Node, np.ndarray] = {}
        if models0 and fresh:
            prog, kept = compile_sets([[k] for k in fresh])
            if kept:
                _, _, b, _ = self.device.eval_bits(prog, self._pool(models0, prog))
                self.device_evals += len(kept) * len(models0)
                self.launches += 1
                for row, k in enumerate(kept):
                    bits[fresh[k]] = b[row]
        out = []
        for k in keys:
            hit, val = self._memo_get(k)
            if hit:
                out.append(val)
                continue
            result = False
            b = bits.get(k)
            if b is not None:
                for m in reversed(self.model_cache.lru_cache.keys()):   # current MRU order
                    p = pos0.get(id(m))
                    if p is not None and (int(b[p >> 6]) >> (p & 63)) & 1:
                        result = self._select(m)
                        break
            self._memo_put(k, result)
            out.append(result)
        return out


def _complement(c: Node) -> Optional[Node]:
    """The conjunct whose truth is the negation of c's under every model, when
    the expression layer builds one: not(X) / X, and eq(a, b) / distinct(a, b)
    (a JUMPI's two branch conditions on a bit-vector word)."""
    if c.op == "not" and len(c.args) == 1:
        return c.args[0]
    if c.op in ("eq", "distinct") and len(c.args) == 2:
        return Node("distinct" if c.op == "eq" else "eq", 1, c.args, c.param)
    return None


def _conjuncts(key: Node) -> List[Node]:
    """The leaf conjuncts of a Bool term (nested ``and`` nodes flattened, each
    distinct conjunct once, in first-seen order)."""
    out: "OrderedDict[Node, None]" = OrderedDict()
    stack = [key]
    while stack:
        n = stack.pop()
        if n.op == "and":
            stack.extend(reversed(n.args))
        elif n is not TRUE:
            out[n] = None
    return list(out)


def _view(model, key: Optional[Node]) -> Dict[str, object]:
    """The assignment ``model.eval(key, model_completion=True)`` evaluates
    under (support_utils.py:65: quick-sat evals the conjunction on the cached
    model): per Model.eval, the first internal model declaring the key's
    declaration, else the last."""
    if isinstance(model, Model):
        m = model.view(key) if key is not None else (model.raw[-1] if model.raw else None)
        return m.assignment if m is not None else {}
    return model.assignment


model_cache = ModelCache()


# ------------------------------------------------------------------ get_model
class _Args:
    """support/support_args.py:5-25 (the fields this core reads): solver timeout
    in ms (get_model), pruning factor (svm.py:319-326 fork filter), the SMT2
    query log directory (support/model.py:62-73)."""
    solver_timeout = 10000
    pruning_factor = 1
    solver_log = None
    unconstrained_storage = False


args = _Args()


class TimeHandler:
    """laser/ethereum/time_handler.py: remaining analysis time in ms."""

    def __init__(self):
        self._start = None
        self._timeout = None

    def start_execution(self, timeout: int):
        self._start = int(time.time() * 1000)
        self._timeout = timeout * 1000

    def time_remaining(self) -> int:
        if self._start is None:
            return 1 << 62
        return self._timeout - (int(time.time() * 1000) - self._start)


time_handler = TimeHandler()


def _no_backend(constraints, minimize, maximize, timeout):
    """The built-in backend: decides only what needs no search.  A set whose
    conjunction folds to True is sat with the empty model (what z3's
    Optimize.check returns for it, support/model.py:76-78), one that folds to
    False is unsat; anything else needs a real SMT backend."""
    root = And(*[c for c in constraints if isinstance(c, Bool)]).raw
    if root is TRUE and not minimize and not maximize:
        return Model([ModelRef({})])
    if root.op == "const" and root.param == 0:
        raise UnsatError
    if not minimize and not maximize:
        witness = _keccak_witness()
        if witness is not None and witness.eval(root, model_completion=True).param == 1:
            return Model([witness])
    raise SolverBackendMissing(
        "quick-sat found no satisfying model and no SMT backend is installed (z3 is absent "
        "in this image): install one with mythril_amd.smt.solver.set_solver_backend()")


def _keccak_witness() -> Optional[ModelRef]:
    """The model the keccak axioms of concrete inputs admit by construction
    (keccak_function_manager.py:116-130: f(c) == keccak(c) and inverse(f(c)) == c):
    keccak256_N and its inverse interpreted exactly at the registered points,
    every variable 0.  Sound: the caller keeps it only if it satisfies the whole
    query.  None when there are no registrations."""
    from .keccak_manager import keccak_function_manager as km
    from .program import FuncInterp
    if not km.concrete_hashes:
        return None
    fn: Dict[str, FuncInterp] = {}
    for data, h in km.concrete_hashes.items():
        n = data.size()
        f = fn.setdefault(f"keccak256_{n}", FuncInterp(0, {}))
        inv = fn.setdefault(f"keccak256_{n}-1", FuncInterp(0, {}))
        f.entries[(data.value,)] = h.value
        inv.entries[(h.value,)] = data.value
    return ModelRef(fn)


solver_backend: Callable = _no_backend


def set_solver_backend(fn: Callable) -> None:
    global solver_backend
    solver_backend = fn
    get_model.cache_clear()


@lru_cache(maxsize=2 ** 23)
def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True,
              solver_timeout=None):
    timeout = solver_timeout or args.solver_timeout
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
        if timeout <= 0:
            raise UnsatError
    for constraint in constraints:
        if type(constraint) == bool and not constraint:
            raise UnsatError
    if type(constraints) != tuple:
        constraints = constraints.get_all_constraints()
    constraints = [c for c in constraints if type(c) != bool]
    if len(maximize) + len(minimize) == 0:
        key = simplify(And(*constraints)).raw
        model_cache.stats["queries"] += 1
        ret_model = model_cache.check_quick_sat(key)
        if ret_model:
            model_cache.stats["lru_hits"] += 1
            return ret_model
        if _seeds_first():
            # no solver that can refute: a seed model of the query is what the
            # backend would return (the SAT-only backend searches from them)
            seed = model_cache.check_seeds(key)
            if seed is not None:
                model_cache.stats["seed_hits"] += 1
                model_cache.put(seed, 1)
                return seed
        model_cache.stats["misses"] += 1
    if args.solver_log:
        from .smtlib import log_query, to_smt2
        log_query(args.solver_log, to_smt2(constraints, minimize, maximize))
    fut = _speculative.pop(_spec_key(constraints, minimize, maximize), None)
    try:
        model = fut.result() if fut is not None else solver_backend(constraints, minimize, maximize, timeout)
    except SolverTimeOutException:
        # a real solver timed out: the reference prunes here (constraints.py:
        # 35-38).  A witness seed that satisfies the query keeps the path
        # instead -- a divergence from the reference, counted
        if not minimize and not maximize and not _seeds_first():
            seed = model_cache.check_seeds(simplify(And(*constraints)).raw)
            if seed is not None:
                model_cache.stats["divergences"] += 1
                model_cache.put(seed, 1)
                return seed
        raise
    model_cache.put(model, 1)
    return model


def _seeds_first() -> bool:
    """Witness seeds are consulted before the backend only when the backend
    cannot refute anything (the built-in one, or the SAT-only search, which
    starts from the seeds itself).  With a real SMT backend installed the
    backend answers first, as the reference's z3 does, so the models that
    reach the LRU -- and later quick-sat choices (arbitrary_jump.py:29-40) --
    are the backend's."""
    return solver_backend is _no_backend or bool(getattr(solver_backend, "uses_seeds", False))


# ------------------------------------------------------------------ fallback pool
_speculative: Dict = {}


def _spec_key(constraints, minimize=(), maximize=()):
    return (tuple(_raw(c) for c in constraints), tuple(minimize), tuple(maximize))


def get_models(queries: Sequence, solver_timeout=None, workers: int = 8) -> List[object]:
    """[get_model(q) for q in queries] with the SMT backend calls overlapped:
    every query's backend call starts up front on a thread pool (speculation),
    then the queries are answered strictly in order, exactly as the sequential
    loop would (quick-sat against the cache as earlier answers left it, memo,
    LRU moves, backend models cached in order); a speculative answer is used
    only where the sequential loop reaches the backend, and discarded
    otherwise.  Each element is a model or the exception get_model raised."""
    from concurrent.futures import ThreadPoolExecutor
    timeout = solver_timeout or args.solver_timeout
    prepared = []
    for q in queries:
        cs = q.get_all_constraints() if hasattr(q, "get_all_constraints") else list(q)
        prepared.append([c for c in cs if type(c) != bool])
    out: List[object] = []
    if not getattr(solver_backend, "speculative", True):
        # a backend that drives the device itself (kernel 2 in the SAT search and
        # the exact procedure's re-check) runs in the sequential loop's thread:
        # one library context is used from one host thread at a time (mythgpu.h)
        for q in queries:
            try:
                out.append(get_model(q if isinstance(q, Constraints) else tuple(q), solver_timeout=solver_timeout))
            except (UnsatError, SolverTimeOutException, SolverBackendMissing) as e:
                out.append(e)
        return out
    with ThreadPoolExecutor(max_workers=max(1, workers)) as pool:
        for cs in prepared:
            key = _spec_key(cs)
            if key not in _speculative:
                _speculative[key] = pool.submit(_safe_backend, cs, timeout)
        try:
            for q in queries:
                try:
                    out.append(get_model(q if isinstance(q, Constraints) else tuple(q),
                                         solver_timeout=solver_timeout))
                except (UnsatError, SolverTimeOutException, SolverBackendMissing) as e:
                    out.append(e)
        finally:
            for cs in prepared:
                _speculative.pop(_spec_key(cs), None)
    return out


def _safe_backend(constraints, timeout):
    """Speculative backend call: exceptions travel to the sequential replay."""
    return solver_backend(constraints, (), (), timeout)


# ------------------------------------------------------------------ Constraints
def _keccak_conditions():
    from .keccak_manager import keccak_function_manager
    return keccak_function_manager.create_conditions()


def query_raw(all_constraints) -> Node:
    """The conjunction get_model's quick-sat evaluates for a constraint list
    (support/model.py:48-56): And of every non-bool constraint."""
    return simplify(And(*[c for c in all_constraints if type(c) != bool])).raw


class Constraints(list):
    def __init__(self, constraint_list: Optional[List] = None):
        super().__init__(self._get_smt_bool_list(constraint_list or []))

    def is_possible(self, solver_timeout=None) -> bool:
        try:
            get_model(self, solver_timeout=solver_timeout)
        except SolverTimeOutException:
            return solver_timeout is not None
        except UnsatError:
            return False
        return True

    def get_model(self, solver_timeout=None):
        try:
            return get_model(self, solver_timeout=solver_timeout)
        except (SolverTimeOutException, UnsatError):
            return None

    def append(self, constraint) -> None:
        constraint = simplify(constraint) if isinstance(constraint, Bool) else \
            symbol_factory.Bool(constraint)
        super().append(constraint)

    @property
    def as_list(self) -> List[Bool]:
        return self[:] + [_keccak_conditions()]

    def get_all_constraints(self):
        return self[:] + [_keccak_conditions()]

    def __copy__(self) -> "Constraints":
        return Constraints(super().copy())

    def copy(self) -> "Constraints":
        return self.__copy__()

    def __deepcopy__(self, memodict=None) -> "Constraints":
        return Constraints(list(self))

    def __add__(self, constraints) -> "Constraints":
        return Constraints(list(self) + self._get_smt_bool_list(constraints))

    def __iadd__(self, constraints: Iterable) -> "Constraints":
        super().__iadd__(self._get_smt_bool_list(constraints))
        return self

    @staticmethod
    def _get_smt_bool_list(constraints: Iterable) -> List[Bool]:
        return [c if isinstance(c, Bool) else symbol_factory.Bool(c) for c in constraints]

    def __hash__(self):
        return tuple(self[:]).__hash__()

    def __eq__(self, other):
        return isinstance(other, list) and len(self) == len(other) and all(
            _raw(a) is _raw(b) for a, b in zip(self, other))


class SnapshotConstraints(Constraints):
    """A path's constraints with the keccak conjunct as it was when the query
    was posed (a fork filter evaluated later in a batch sees the function
    manager of its own time); hashed and compared as the plain Constraints, so
    get_model's cache is shared with them."""

    def __init__(self, constraint_list, keccak_conjunct):
        super().__init__(list(constraint_list))
        self._kc = keccak_conjunct

    def get_all_constraints(self):
        return self[:] + [self._kc]

    @property
    def as_list(self):
        return self.get_all_constraints()

    __hash__ = Constraints.__hash__
