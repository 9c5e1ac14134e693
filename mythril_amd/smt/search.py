"""SAT-only SMT backend: kernel 2 as a model finder.

The reference hands every quick-sat miss to z3 (support/model.py:56-82).  No
SMT solver exists in this image, so this backend answers the way SURVEY §8(b)
allows a prefilter to answer: SAT with a model, or not at all.  It never claims
UNSAT: a query it cannot satisfy raises ``SolverBackendMissing`` (callers that
keep unknown paths, ``LaserEVM.unknown_forks = "keep"``, keep them; issue
confirmation counts them as unconfirmed).

Where a model comes from, in order:

1. the witness seeds of the model cache (laser/witness.py), evaluated on
   kernel 2;
2. a guided search: the seeds that satisfy the most conjuncts are repaired,
   one unsatisfied conjunct at a time, by *inverting* the conjunct toward true
   (propagation-based local search for bit-vectors: the value a sub-term must
   take is pushed down through the operators -- add/sub/xor/not by the other
   operand, division and remainder by a constant over all residues, extract /
   concat / zero-extend by bit slices, compares to the neighbouring value,
   ``ite`` through its taken arm or its condition, ``select`` to an entry of
   the array or to the index of one of its stores -- until it names a variable
   or an array entry, which is then assigned).  Every repaired candidate is
   completed so the function managers' axioms hold (keccak256_N and its
   inverse, Power) and the whole batch of candidates is scored on kernel 2
   (one launch: every conjunct x every candidate, per-conjunct bitmaps); the
   best are repaired again for a few rounds.
3. minimised terms (get_transaction_sequence's calldata sizes and call values,
   analysis/solver.py:219-259) are lowered afterwards by a batched descent --
   a local minimum, not z3 Optimize's global one.

A model is returned only when kernel 2 found it satisfying every conjunct of
the query; the host does not decide satisfaction anywhere.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .expr import TRUE, Node
from .program import ArrayInterp, FuncInterp, PoolColumns
from .semantics import apply_op
from .refute import refutes
from .solver import Model, ModelRef, SolverBackendMissing, UnsatError, _conjuncts, query_raw

M256 = (1 << 256) - 1


def _mask(w: int) -> int:
    return (1 << w) - 1


class _Eval:
    """Values of the terms of a query under one assignment (model completion:
    absent variables 0, arrays and functions their default / else value)."""

    def __init__(self, assign: Dict[str, object]):
        self.a = assign
        self.memo: Dict[int, object] = {}

    def arr(self, node: Node):
        got = self.memo.get(id(node))
        if got is not None:
            return got
        if node.op == "array":
            it = self.a.get(node.param[0])
            out = (it.default, it.entries) if isinstance(it, ArrayInterp) else (0, {})
        elif node.op == "K":
            out = (self(node.args[0]), {})
        elif node.op == "store":
            d, e = self.arr(node.args[0])
            out = (d, {**e, self(node.args[1]): self(node.args[2])})
        else:
            raise ValueError(node.op)
        self.memo[id(node)] = out
        return out

    def __call__(self, node: Node) -> int:
        got = self.memo.get(id(node))
        if got is not None:
            return got
        op = node.op
        if op == "const":
            out = node.param
        elif op == "var":
            v = self.a.get(node.param, 0)
            out = v if isinstance(v, int) else 0
        elif op == "select":
            d, e = self.arr(node.args[0])
            out = e.get(self(node.args[1]), d)
        elif op == "uf":
            it = self.a.get(node.param[0])
            key = tuple(self(x) for x in node.args)
            out = it.entries.get(key, it.else_value) if isinstance(it, FuncInterp) else 0
        else:
            out = apply_op(op, node.width, [self(x) for x in node.args], [x.width for x in node.args], node.param)
        self.memo[id(node)] = out
        return out


# a repair: {name: int} for variables, {(name, index): int} for array entries
Repair = Dict[object, int]


class _Inverter:
    """Values that make a term take a target value under one assignment."""

    LIMIT = 48           # repairs returned per call

    def __init__(self, ev: _Eval, rng: np.random.Generator):
        self.ev = ev
        self.rng = rng
        # (term, target) -> repairs: the terms are hash-consed DAGs, so one query
        # reaches a subterm from many parents; its repairs under this assignment
        # do not depend on the path that reached it (the first one computed is kept)
        self.memo: Dict[Tuple[int, int], List[Repair]] = {}

    def bool_true(self, node: Node) -> List[Repair]:
        return self.inv(node, 1)[: self.LIMIT]

    def inv(self, n: Node, t: int, depth: int = 0) -> List[Repair]:
        if depth > 40:
            return []
        # a result computed near the depth cut may be truncated: the memo keeps
        # it only for visits as deep (coarse buckets of 10), so a shallower visit
        # of the same subterm computes its own
        key = (id(n), t, depth // 10)
        got = self.memo.get(key)
        if got is None:
            got = self.memo[key] = self._inv(n, t, depth)[: 4 * self.LIMIT]
        return got

    def _inv(self, n: Node, t: int, depth: int) -> List[Repair]:
        ev = self.ev
        w = n.width
        t &= _mask(w) if w else M256
        if ev(n) == t:
            return [{}]
        op, a = n.op, n.args
        d = depth + 1
        if op == "var":
            return [{n.param: t}]
        if op == "const":
            return []
        if op == "not":
            return self.inv(a[0], 1 - t, d)
        if op == "and":
            if t:
                return self._all(a, [1] * len(a), d)
            return self._any(a, [0] * len(a), d)
        if op == "or":
            if t:
                return self._any(a, [1] * len(a), d)
            return self._all(a, [0] * len(a), d)
        if op == "implies":
            return self.inv(a[0], 0, d) + self.inv(a[1], 1, d) if t else self._all(a, [1, 0], d)
        if op in ("eq", "distinct"):
            want_eq = (t == 1) == (op == "eq")
            x, y = a
            vx, vy = ev(x), ev(y)
            if want_eq:
                return self.inv(x, vy, d) + self.inv(y, vx, d)
            m = _mask(x.width)
            return self.inv(x, (vy + 1) & m, d) + self.inv(y, (vx + 1) & m, d) + self.inv(x, vy ^ 1, d)
        if op in _CMP:
            return self._cmp(n, t, d)
        if op == "ite":
            c, x, y = a
            if ev(c):
                out = self.inv(x, t, d)
                if ev(y) == t:
                    out += self.inv(c, 0, d)
            else:
                out = self.inv(y, t, d)
                if ev(x) == t:
                    out += self.inv(c, 1, d)
            return out
        if op in ("bvadd", "bvsub", "bvxor"):
            x, y = a
            m = _mask(w)
            vx, vy = ev(x), ev(y)
            if op == "bvadd":
                return self.inv(x, (t - vy) & m, d) + self.inv(y, (t - vx) & m, d)
            if op == "bvsub":
                return self.inv(x, (t + vy) & m, d) + self.inv(y, (vx - t) & m, d)
            return self.inv(x, t ^ vy, d) + self.inv(y, t ^ vx, d)
        if op == "bvnot":
            return self.inv(a[0], ~t & _mask(w), d)
        if op == "bvneg":
            return self.inv(a[0], -t & _mask(w), d)
        if op in ("bvand", "bvor"):
            x, y = a
            out = []
            for p, q in ((x, y), (y, x)):
                vq = ev(q)
                if op == "bvand" and t & ~vq & _mask(w) == 0:
                    out += self.inv(p, (ev(p) & ~vq) | t, d)
                if op == "bvor" and vq & ~t & _mask(w) == 0:
                    out += self.inv(p, (ev(p) & vq) | (t & ~vq), d)
            return out
        if op == "bvmul":
            x, y = a
            out = []
            for p, q in ((x, y), (y, x)):
                c = ev(q)
                if c & 1:
                    out += self.inv(p, t * pow(c, -1, 1 << w) & _mask(w), d)
                elif c and t % (c & -c) == 0:
                    k = (c & -c).bit_length() - 1
                    out += self.inv(p, (t >> k) * pow(c >> k, -1, 1 << w) & _mask(w), d)
            return out
        if op in ("bvudiv", "bvurem") and a[1].op == "const" and a[1].param:
            c = a[1].param
            x = a[0]
            vx = ev(x)
            if op == "bvudiv":
                if t * c > _mask(w):
                    return []
                residues = list(range(c)) if c <= 64 else sorted({0, vx % c, c - 1,
                                                                  int(self.rng.integers(0, min(c, 1 << 62)))})
                out = []
                for r in residues:
                    out += self.inv(x, t * c + r, d)
                return out
            if t >= c:
                return []
            return self.inv(x, (vx - vx % c) + t, d) + self.inv(x, t, d)
        if op == "bvudiv":
            # a divisor that is not a constant (an uninterpreted Power, say):
            # the numerator for the divisor's current value
            x, y = a
            vx, vy = ev(x), ev(y)
            if vy == 0 or t * vy > _mask(w):
                return []
            out = []
            for r in sorted({0, vx % vy, vy - 1}):
                out += self.inv(x, t * vy + r, d)
            return out
        if op == "bvurem":
            x, y = a
            vx, vy = ev(x), ev(y)
            if vy == 0 or t >= vy:
                return []
            return self.inv(x, (vx - vx % vy) + t, d)
        if op in ("bvshl", "bvlshr") and a[1].op == "const":
            k = a[1].param
            x = a[0]
            if k >= w:
                return []
            if op == "bvshl":
                if t & _mask(k):
                    return []
                return self.inv(x, (t >> k) | (ev(x) & (_mask(k) << (w - k))), d)
            if t >> (w - k) if k else 0:
                return []
            return self.inv(x, (t << k) | (ev(x) & _mask(k)), d)
        if op == "concat":
            parts, lo, tgt = [], w, []
            for x in a:
                lo -= x.width
                tgt.append((t >> lo) & _mask(x.width))
                parts.append(x)
            return self._all(parts, tgt, d, merge_last=True)
        if op == "extract":
            hi, lo = n.param
            x = a[0]
            vx = ev(x)
            field = _mask(hi - lo + 1) << lo
            return self.inv(x, (vx & ~field) | (t << lo), d)
        if op == "zero_extend":
            x = a[0]
            return self.inv(x, t, d) if t <= _mask(x.width) else []
        if op == "sign_extend":
            x = a[0]
            return self.inv(x, t & _mask(x.width), d)
        if op == "select":
            return self._select(n, t, d)
        if op in ("bvadd_noovfl_u", "bvsub_noudfl_u", "bvumul_noovfl"):
            return self._overflow(op, a, t, d)
        if op == "uf":
            return self._uf(n, t, d)
        return []

    def _uf(self, n: Node, t: int, d: int) -> List[Repair]:
        """f(args) := t for an uninterpreted function (keccak256_N, Power): the
        interpretation holds no free choice (complete() rebuilds it from the
        axioms), but another application with value t does -- move the
        arguments to that application's key (a mapping slot keyed by a sender
        made equal to one keyed by a calldata address, say)."""
        it = self.ev.a.get(n.param[0])
        if not isinstance(it, FuncInterp):
            return []
        out: List[Repair] = []
        for key, v in it.entries.items():
            if v == t and len(key) == len(n.args):
                out += self._all(list(n.args), list(key), d)
                if len(out) >= self.LIMIT:
                    break
        return out

    def _overflow(self, op: str, a, t: int, d: int) -> List[Repair]:
        """The unsigned overflow predicates (bitvec_helper.py:200-246):
        bvadd_noovfl_u(x, y) = x + y < 2^w, bvsub_noudfl_u(x, y) = y <= x,
        bvumul_noovfl(x, y) = x * y < 2^w; t = 0 asks for the overflow."""
        x, y = a
        w = x.width
        m = _mask(w)
        vx, vy = self.ev(x), self.ev(y)
        out: List[Repair] = []
        if op == "bvadd_noovfl_u":
            if t:
                return self.inv(x, m - vy, d) + self.inv(y, m - vx, d) + self.inv(x, 0, d)
            if vy:
                out += self.inv(x, (1 << w) - vy, d) + self.inv(x, m, d)
            if vx:
                out += self.inv(y, (1 << w) - vx, d) + self.inv(y, m, d)
            return out or self.inv(x, m, d)
        if op == "bvsub_noudfl_u":
            if t:
                return self.inv(x, vy, d) + self.inv(y, vx, d) + self.inv(y, 0, d)
            if vy:
                out += self.inv(x, vy - 1, d) + self.inv(x, 0, d)
            if vx < m:
                out += self.inv(y, vx + 1, d) + self.inv(y, m, d)
            return out
        if t:
            out = self.inv(x, 0, d) + self.inv(y, 0, d)
            if vy:
                out += self.inv(x, m // vy, d)
            return out
        if vy:
            out += self.inv(x, min(m, -(-(1 << w) // vy)), d)
        if vx:
            out += self.inv(y, min(m, -(-(1 << w) // vx)), d)
        return out + self.inv(x, m, d)

    # -- helpers ----------------------------------------------------------------------
    def _any(self, args, targets, d) -> List[Repair]:
        out: List[Repair] = []
        for x, t in zip(args, targets):
            if self.ev(x) != t:
                out += self.inv(x, t, d)
            if len(out) >= self.LIMIT:
                break
        return out

    def _all(self, args, targets, d, merge_last: bool = False) -> List[Repair]:
        """One repair making every arg take its target: the per-arg repairs
        merged (each arg's first option; later args win conflicts, which is
        what a calldata word's ascending byte conditions need), plus, for
        variety, the per-arg alternatives of the first wrong arg."""
        merged: Repair = {}
        first_alts: List[Repair] = []
        for x, t in zip(args, targets):
            if self.ev(x) == t:
                continue
            opts = self.inv(x, t, d)
            if not opts:
                return []
            if not first_alts:
                first_alts = opts[1:8]
            merged.update(opts[0])
        return [merged] + [{**merged, **alt} for alt in first_alts]

    def _cmp(self, n: Node, t: int, d: int) -> List[Repair]:
        op, (x, y) = n.op, n.args
        w = x.width
        m = _mask(w)
        vx, vy = self.ev(x), self.ev(y)
        signed = op in ("bvslt", "bvsle", "bvsgt", "bvsge")
        if not t:
            op = _NEG[op]
        # normalise to x < y, x <= y
        if op in ("bvugt", "bvsgt", "bvuge", "bvsge"):
            x, y, vx, vy = y, x, vy, vx
            op = {"bvugt": "bvult", "bvsgt": "bvslt", "bvuge": "bvule", "bvsge": "bvsle"}[op]
        strict = op in ("bvult", "bvslt")
        lo_y = vy - 1 if strict else vy          # x := something <= lo_y
        hi_x = vx + 1 if strict else vx          # y := something >= hi_x
        out: List[Repair] = []
        if signed:
            half = 1 << (w - 1)
            sy = vy - (1 << w) if vy >= half else vy
            sx = vx - (1 << w) if vx >= half else vx
            if (sy - 1 if strict else sy) >= -half:
                out += self.inv(x, (sy - 1 if strict else sy) & m, d)
                out += self.inv(x, 0, d) if 0 <= (sy - 1 if strict else sy) else []
            if (sx + 1 if strict else sx) < half:
                out += self.inv(y, (sx + 1 if strict else sx) & m, d)
        else:
            if lo_y >= 0:
                out += self.inv(x, lo_y, d)
                if lo_y > 0:
                    out += self.inv(x, 0, d)
            if hi_x <= m:
                out += self.inv(y, hi_x, d)
                out += self.inv(y, m, d)
        return out

    def _select(self, n: Node, t: int, d: int) -> List[Repair]:
        """select(array, index) := t: set the array's entry at the index's value
        (through the store chain to the base) or move the index to a store key
        whose value is t -- or to any store key (the caller's target may only be
        a guess, e.g. below an uninterpreted divisor)."""
        arr, idx = n.args
        vi = self.ev(idx)
        out: List[Repair] = []
        a = arr
        keys: List[Tuple[Node, Node]] = []
        while a.op == "store":
            keys.append((a.args[1], a.args[2]))
            a = a.args[0]
        hit = next(((k, v) for k, v in keys if self.ev(k) == vi), None)
        if hit is not None:
            out += self.inv(hit[1], t, d)
        elif a.op == "array":
            out.append({(a.param[0], vi): t})
        for k, v in keys:
            kv = self.ev(k)
            if kv != vi and (self.ev(v) == t or len(out) < 4):
                out += self.inv(idx, kv, d)
                if self.ev(v) == t:
                    out += self.inv(k, vi, d)          # or the store's key to the index
        return out


_CMP = {"bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge"}
_NEG = {"bvult": "bvuge", "bvule": "bvugt", "bvugt": "bvule", "bvuge": "bvult",
        "bvslt": "bvsge", "bvsle": "bvsgt", "bvsgt": "bvsle", "bvsge": "bvslt"}


def apply_repair(assign: Dict[str, object], rep: Repair) -> Dict[str, object]:
    out = dict(assign)
    for k, v in rep.items():
        if isinstance(k, tuple):
            name, idx = k
            it = out.get(name)
            base = it if isinstance(it, ArrayInterp) else ArrayInterp(0, {})
            new = ArrayInterp(base.default, base.entries)
            new.entries[idx] = v
            out[name] = new
        else:
            out[k] = v
    return out


class _Completed(dict):
    """A completed assignment, with the value complete() gave each registered
    keccak input (`kvals`): a candidate one repair away reuses the values of
    the inputs the repair does not reach."""
    __slots__ = ("kvals",)


_DEPS: Dict[int, Tuple[Node, frozenset, bool]] = {}
_DEPS_MAX = 1 << 16          # entries keep their terms alive: bounded, cleared on keccak reset


def clear_deps() -> None:
    _DEPS.clear()


def _deps(raw: Node) -> Tuple[frozenset, frozenset]:
    """(variable and array names a term reads, the uninterpreted functions it
    applies -- whose interpretations complete() rebuilds)."""
    got = _DEPS.get(id(raw))
    if got is not None and got[0] is raw:
        return got[1], got[2]
    names, uf, seen, stack = set(), set(), set(), [raw]
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        if n.op == "var":
            names.add(n.param)
        elif n.op == "array":
            names.add(n.param[0])
        elif n.op == "uf":
            uf.add(n.param[0])
        stack.extend(n.args)
    fs, fu = frozenset(names), frozenset(uf)
    if len(_DEPS) >= _DEPS_MAX:
        _DEPS.clear()
    _DEPS[id(raw)] = (raw, fs, fu)
    return fs, fu


def _changed(rep: Repair) -> frozenset:
    return frozenset(k if isinstance(k, str) else k[0] for k in rep)


def complete(assign: Dict[str, object], base: Optional[_Completed] = None,
             changed: frozenset = frozenset()) -> _Completed:
    """The function managers' interpretations under `assign`, rebuilt so their
    axioms hold (keccak_function_manager.py:116-179, exponent_function_manager
    .py:32-60): keccak256_N at every registered input's value (the concrete hash
    of a registered concrete input, else the k-th multiple of 64 in N's
    interval) with its inverse, Power at the concrete points and at every
    symbolic EXP's value (base 256: the 256**(e % 32) its periodicity axiom
    demands; other bases: the power when it is positive, else 1)."""
    from .exponent_manager import exponent_function_manager as em
    from .keccak_manager import PART, keccak_function_manager as km
    out = _Completed((k, v) for k, v in assign.items() if not k.startswith("keccak256_") and k != "Power")
    ev = _Eval(out)
    prev = base.kvals if isinstance(base, _Completed) else None
    kvals: Dict[Node, int] = {}
    concrete = {(c.size(), c.value): h.value for c, h in km.concrete_hashes.items()}
    tabs: Dict[str, FuncInterp] = {}
    for (n, cv), h in concrete.items():
        tabs.setdefault(f"keccak256_{n}", FuncInterp(0, {})).entries[(cv,)] = h
        tabs.setdefault(f"keccak256_{n}-1", FuncInterp(0, {})).entries[(h,)] = cv
    km.assign_intervals()               # intervals in the reference's order
    fresh: Dict[int, int] = {}
    for n, xs in km.symbolic_inputs.items():
        f = tabs.setdefault(f"keccak256_{n}", FuncInterp(0, {}))
        inv = tabs.setdefault(f"keccak256_{n}-1", FuncInterp(0, {}))
        for x in dict.fromkeys(x.raw for x in xs):      # registered once per SHA3 executed
            v = prev.get(x) if prev is not None else None
            if v is not None:
                # the base's value stands unless the input reads a changed name or
                # an uninterpreted function the assignment interprets (during this
                # loop `out` holds no keccak / Power tables: ev gives their
                # applications the completion value, as it did for the base)
                names, ufs = _deps(x)
                if (names & changed) or (ufs & changed) or any(u in out for u in ufs):
                    v = None
            if v is None:
                v = ev(x)
            kvals[x] = v
            if (v,) in f.entries:
                continue
            h = concrete.get((n, v))
            if h is None:
                k = fresh.get(n, 0)
                fresh[n] = k + 1
                lo = km.interval_hook_for_size.get(n, 0) * PART
                h = (lo + 63) // 64 * 64 + 64 * k
            f.entries[(v,)] = h
            inv.entries[(h,)] = v
    pw = FuncInterp(0, dict(em.concrete_points))
    for base, exponent in em.symbolic_points:
        b, e = ev(base.raw), ev(exponent.raw)
        if b == 256:
            v = 256 ** (e % 32)
        else:
            v = pow(b, e, 1 << 256)
            v = v if 0 < v < 1 << 255 else 1
        pw.entries.setdefault((b, e), v)
    out.update(tabs)
    out["Power"] = pw
    out.kvals = kvals
    return out


def _model(assign: Dict[str, object]) -> Model:
    ref = ModelRef()
    ref.assignment = assign
    return Model([ref])


class SatSearchBackend:
    """``solver.set_solver_backend(SatSearchBackend(model_cache))``: answers
    get_model's misses with a model found on kernel 2, or raises
    SolverBackendMissing (unknown).  With ``exact`` (an exact.ExactSolver) the
    queries the refutations, the seeds and the search leave open go to the
    exact decision procedure: a model (re-checked on kernel 2), UnsatError, or
    SolverTimeOutException when its budget runs out -- z3's three answers in
    support/model.py:37-82, so nothing stays "unknown"."""

    uses_seeds = True          # get_model consults the seeds before calling it
    speculative = False        # it launches kernel 2: never from get_models' worker threads

    def __init__(self, cache, search: bool = True, rounds: int = 12, beam: int = 6,
                 max_candidates: int = 4096, patience: int = 3, seed: int = 0x5EA5C4,
                 exact=None, exact_ms: int = 60000):
        self.cache = cache
        self.search = search
        self.exact = exact
        self.exact_ms = exact_ms
        self.rounds = rounds
        self.beam = beam
        self.max_candidates = max_candidates
        self.patience = patience       # rounds without a better best count before giving up
        self.rng = np.random.default_rng(seed)
        # completed assignments by the assignment's identity: an LRU bounded by
        # the model cache plus the seeds (each entry holds the
        # completed dict with its keccak and Power tables)
        self._memo_completed: "OrderedDict[int, tuple]" = OrderedDict()
        self._memo_cap = 2048
        self._start_cols: Optional[tuple] = None      # (the starting pool's assignments, their PoolColumns)
        self.stats: Dict[str, int] = {"calls": 0, "refuted": 0, "seed": 0, "search": 0, "unknown": 0,
                                      "candidates": 0, "launches": 0, "minimised": 0,
                                      "exact_sat": 0, "exact_unsat": 0, "exact_timeout": 0}

    def __call__(self, constraints, minimize, maximize, timeout):
        self.stats["calls"] += 1
        key = query_raw(constraints)
        if refutes(_conjuncts(key)):
            self.stats["refuted"] += 1
            raise UnsatError
        model = self.cache.check_seeds(key)
        if model is not None:
            self.stats["seed"] += 1
        elif self.search:
            model = self._search(key)
            if model is not None:
                self.stats["search"] += 1
        if model is None and self.exact is not None:
            return self._decide(key, minimize, timeout)
        if model is None:
            self.stats["unknown"] += 1
            raise SolverBackendMissing("SAT-only backend: no candidate model satisfies the query (unknown)")
        if minimize:
            model = self._minimise(key, model, minimize)
        return model

    def _decide(self, key: Node, minimize, timeout) -> Model:
        """The exact procedure on a query the cheaper answers left open."""
        from .solver import SolverTimeOutException
        conj = [c for c in _conjuncts(key) if c is not TRUE]
        budget = int(self.exact_ms)         # the wall-clock guard; the budget proper is conflicts
        mins = [m.raw if hasattr(m, "raw") else m for m in minimize]
        st, assign = self.exact.check(conj, mins, max_ms=max(budget, 1))
        if st == "unsat":
            self.stats["exact_unsat"] += 1
            raise UnsatError
        if st == "unknown":
            self.stats["exact_timeout"] += 1
            raise SolverTimeOutException
        self.stats["exact_sat"] += 1
        # every model is checked by kernel 2 before anyone sees it (a conjunct
        # kernel 2 has no row for: by the host evaluator); a session's model
        # that fails is decided again alone, and a second failure is a bug
        live = [c for c in conj if c.op != "const"]
        for attempt in range(2):
            if not live or self._holds(live, assign):
                return _model(assign)
            if attempt:
                break
            self.stats["exact_recheck"] = self.stats.get("exact_recheck", 0) + 1
            st, assign = self.exact.check(conj, mins, max_ms=max(budget, 1), fresh=True)
            if st == "unsat":
                raise RuntimeError("the exact procedure answered sat and then unsat on one query")
            if st == "unknown":
                self.stats["exact_timeout"] += 1
                raise SolverTimeOutException
        raise RuntimeError("the exact procedure's model does not satisfy the query on kernel 2")

    def _holds(self, live, assign) -> bool:
        counts, hit = self._score(live, [assign])
        if hit is False:
            ref = ModelRef(assign)
            return all(ref.eval(c, model_completion=True).param == 1 for c in live)
        return hit == 0

    def _completed(self, assign: Dict[str, object]) -> "_Completed":
        """complete(assign), memoised per assignment object while neither it
        (its size) nor the function managers' registrations change: the seeds
        and LRU models start every search, and completing them anew each time
        was most of a search's host time.  (Any candidate is still checked on
        kernel 2 before it is reported, so the memo affects which model is
        found, never whether one is.)"""
        from .exponent_manager import exponent_function_manager as em
        from .keccak_manager import keccak_function_manager as km
        state = (sum(len(v) for v in km.symbolic_inputs.values()), len(km.concrete_hashes),
                 len(em.symbolic_points), len(em.concrete_points), len(assign))
        got = self._memo_completed.get(id(assign))
        if got is not None:
            self._memo_completed.move_to_end(id(assign))
        if got is not None and got[0] is assign and got[1] == state:
            return got[2]
        out = complete(dict(assign))
        self._memo_completed[id(assign)] = (assign, state, out)
        self._memo_completed.move_to_end(id(assign))
        while len(self._memo_completed) > self._memo_cap:
            self._memo_completed.popitem(last=False)
        return out

    def _columns(self, pool: List[Dict[str, object]]) -> PoolColumns:
        """The starting pool's model columns, kept while the pool holds the same
        completed assignments (the memo above returns the same objects until a
        registration or the LRU changes): consecutive searches then serialise only
        the variables they add, not every variable of 1,000+ models again.  A
        completed assignment is never changed after it is made."""
        got = self._start_cols
        if got is None or len(got[0]) != len(pool) or not all(a is b for a, b in zip(got[0], pool)):
            got = self._start_cols = (list(pool), PoolColumns(list(pool)))
        return got[1]

    # -- kernel-2 scoring ---------------------------------------------------------------
    def _score(self, conj: Sequence[Node], assigns: List[Dict[str, object]], columns=None):
        """(per-candidate satisfied-conjunct counts, index of a candidate that
        satisfies every conjunct or None, or False when a conjunct has no
        kernel-2 row: no candidate can then be reported); one kernel-2 launch."""
        models = [_model(a) for a in assigns]
        rows = self.cache.conjunct_rows(list(conj), models, columns)
        self.stats["launches"] += 1
        self.stats["candidates"] += len(models)
        n = len(models)
        counts = np.zeros(n, dtype=np.int64)
        allsat = np.ones(n, dtype=bool)
        idx = np.arange(n)
        self._sat = np.zeros((len(conj), n), dtype=bool)     # conjunct c holds under candidate i
        for k, c in enumerate(conj):
            r = rows.get(c)
            if r is None:                      # not evaluable on the device: no answer
                return counts, False
            bits = ((r[idx >> 6] >> (idx & 63).astype(np.uint64)) & np.uint64(1)).astype(bool)
            self._sat[k] = bits
            counts += bits
            allsat &= bits
        hit = np.flatnonzero(allsat)
        return counts, (int(hit[0]) if hit.size else None)

    def _search(self, key: Node) -> Optional[Model]:
        conj = [c for c in _conjuncts(key) if c.op != "const"]
        if not conj:
            return None
        # start from the models the cache already holds (answers to earlier,
        # usually overlapping queries: a path's prefix, a module's pre-solve),
        # then the seeds
        lru = [m for m in reversed(self.cache.model_cache.lru_cache.keys()) if isinstance(m, Model)]
        seeds = lru + (self.cache._seed_models() or [_model({})])
        pool = [self._completed(m.raw[-1].assignment) for m in seeds]
        counts, hit = self._score(conj, pool, self._columns(pool))
        if hit is False:
            return None                        # a conjunct kernel 2 cannot evaluate
        if hit is not None:
            return _model(pool[hit])
        seen = set()
        best, stall = int(counts.max()), 0
        order = np.argsort(-counts, kind="stable")
        beam = [pool[i] for i in order[: self.beam]]
        # which conjuncts each beam member violates: kernel 2's bitmaps of the
        # launch that scored it (no host evaluation)
        beam_wrong = [[c for k, c in enumerate(conj) if not self._sat[k, i]] for i in order[: self.beam]]
        for _ in range(self.rounds):
            cands: List[Dict[str, object]] = []
            for a, wrong in zip(beam, beam_wrong):
                ev = _Eval(a)
                inv = _Inverter(ev, self.rng)
                firsts: Repair = {}
                for c in wrong:
                    opts = inv.bool_true(c)           # memoised: the loop below reuses them
                    if opts:
                        firsts.update(opts[0])
                if len(wrong) > 1 and firsts:
                    # every wrong conjunct's first repair at once (independent
                    # conjuncts -- a selector, a call value, a sender -- are
                    # usually fixed together)
                    cands.append(complete(apply_repair(a, firsts), a, _changed(firsts)))
                for c in wrong[:4]:
                    for rep in inv.bool_true(c):
                        sig = (id(a), tuple(sorted(map(repr, rep.items()))))
                        if not rep or sig in seen:
                            continue
                        seen.add(sig)
                        cands.append(complete(apply_repair(a, rep), a, _changed(rep)))
                        if len(cands) >= self.max_candidates:
                            break
            if not cands:
                return None
            counts, hit = self._score(conj, cands)
            if hit is False:
                return None
            if hit is not None:
                return _model(cands[hit])
            top = int(counts.max())
            best, stall = (top, 0) if top > best else (best, stall + 1)
            if stall >= self.patience:
                return None                    # no round has come closer: unknown
            order = np.argsort(-counts, kind="stable")
            beam = [cands[i] for i in order[: self.beam]]
            beam_wrong = [[c for k, c in enumerate(conj) if not self._sat[k, i]] for i in order[: self.beam]]
        return None

    # -- minimisation --------------------------------------------------------------------
    def _minimise(self, key: Node, model: Model, minimize) -> Model:
        """Lower each minimised term in turn (calldata size, call value, in the
        order get_transaction_sequence lists them) while the query stays
        satisfied: every candidate value below the current one that the term's
        variable can take is evaluated in one kernel-2 batch and the smallest
        satisfying one is kept."""
        conj = [c for c in _conjuncts(key) if c.op != "const"]
        assign = dict(model.raw[-1].assignment)
        for term in minimize:
            raw = term.raw if hasattr(term, "raw") else term
            if raw.op != "var":
                continue
            cur = _Eval(assign)(raw)
            if cur == 0:
                continue
            vals = sorted({v for v in (0, 1, 2, 3, 4, 32, 36, 64, 68, 100, 132, 164, 196, 228, 260)
                           if v < cur} | {cur - k for k in range(1, min(cur, 64) + 1)} |
                          {cur >> k for k in range(1, 12)})
            cands = [complete({**assign, raw.param: v}, assign, frozenset((raw.param,))) for v in vals]
            counts, hit = self._score(conj, cands)
            if hit is False:
                break
            best = next((i for i in range(len(vals)) if counts[i] == len(conj)), None)
            if best is not None:
                assign = cands[best]
                self.stats["minimised"] += 1
        return _model(assign) if assign is not model.raw[-1].assignment else model
