"""The exact decision procedure behind kernel 2 (include/mythsmt.h, libmythsmt.so).

Kernel 2 (quick-sat over the model cache) and the SAT-only search
(search.py) answer a query with a model or not at all.  The reference
answers what they leave open with z3 (support/model.py:37-82): a model, or
``UnsatError``, or ``SolverTimeOutException`` when the solver gives up --
and ``Constraints.is_possible`` prunes on both of the latter
(state/constraints.py:33-43).  ``ExactSolver`` is that last step here: the
query's conjuncts go to ``ms_solve`` (bit-blasting + CDCL, host C++) as a
post-order node table; the model it returns -- variable values, each array's
point reads, each uninterpreted function's applications -- becomes a
``ModelRef`` assignment the callers (and kernel 2, which re-checks it) read
exactly as they read any other model.  ``minimize`` terms are met
lexicographically, as z3's Optimize does with several objectives
(analysis/solver.py:219-259).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
import time
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

from .expr import Node

PKG_DIR = Path(__file__).resolve().parents[1]
SRC = PKG_DIR / "csrc" / "bvsat.cpp"
HEADER = PKG_DIR.parent / "include" / "mythsmt.h"
LIB_PATH = PKG_DIR / "libmythsmt.so"
HASH_PATH = LIB_PATH.with_name(LIB_PATH.name + ".sha256")
CXX = os.environ.get("CXX", "g++")

# include/mythsmt.h opcodes, by expr.py op name
OPS = {name: i for i, name in enumerate((
    "const", "var", "bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod",
    "bvand", "bvor", "bvxor", "bvnot", "bvneg", "bvshl", "bvlshr", "bvashr",
    "eq", "distinct", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
    "and", "or", "not", "xor", "implies", "ite", "concat", "extract", "zero_extend", "sign_extend",
    "bvadd_noovfl_u", "bvumul_noovfl", "bvsub_noudfl_u", "select", "uf", "array", "K", "store"))}
MS_SAT, MS_UNSAT, MS_UNKNOWN, MS_EINVAL, MS_ESPACE = 1, 0, 2, -1, -2


class MsQuery(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_uint32), ("nodes", ctypes.c_void_p), ("args", ctypes.c_void_p),
                ("limbs", ctypes.c_void_p), ("n_roots", ctypes.c_uint32), ("roots", ctypes.c_void_p),
                ("n_minimize", ctypes.c_uint32), ("minimize", ctypes.c_void_p),
                ("n_vars", ctypes.c_uint32), ("n_arrays", ctypes.c_uint32), ("n_funcs", ctypes.c_uint32)]


class MsLimits(ctypes.Structure):
    _fields_ = [("max_conflicts", ctypes.c_uint64), ("max_ms", ctypes.c_uint32), ("minimize_ms", ctypes.c_uint32)]


class MsStats(ctypes.Structure):
    _fields_ = [("vars", ctypes.c_uint64), ("clauses", ctypes.c_uint64), ("conflicts", ctypes.c_uint64),
                ("decisions", ctypes.c_uint64), ("propagations", ctypes.c_uint64), ("solves", ctypes.c_uint32),
                ("ms", ctypes.c_uint32)]


_SOLVE_ARGS = [ctypes.POINTER(MsQuery), ctypes.POINTER(MsLimits), ctypes.c_void_p, ctypes.c_uint32,
               ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(MsStats)]
SIGNATURES = {
    "ms_abi_version": (ctypes.c_int, []),
    "ms_solve": (ctypes.c_int, _SOLVE_ARGS),
    "ms_session_open": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p)]),
    "ms_session_close": (None, [ctypes.c_void_p]),
    "ms_session_solve": (ctypes.c_int, [ctypes.c_void_p] + _SOLVE_ARGS),
}


def _command(out: str) -> List[str]:
    return [CXX, "-O3", "-std=c++17", "-fPIC", "-shared", str(SRC), "-o", out]


def source_hash() -> str:
    import hashlib
    h = hashlib.sha256()
    for p in (SRC, HEADER):
        h.update(p.name.encode() + b"\0" + p.read_bytes() + b"\0")
    h.update(" ".join(a for a in _command("OUT")[1:] if not a.startswith("/")).encode())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile libmythsmt.so in-tree (host C++, g++ -O2); rebuilt when the
    recorded source hash differs."""
    want = source_hash()
    if not force and LIB_PATH.exists() and HASH_PATH.exists() and HASH_PATH.read_text().strip() == want:
        return LIB_PATH
    cmd = _command(str(LIB_PATH) + ".tmp")
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(str(LIB_PATH) + ".tmp", LIB_PATH)
    HASH_PATH.write_text(want + "\n")
    return LIB_PATH


_lib = None
_lock = threading.Lock()


def load() -> ctypes.CDLL:
    """The in-tree libmythsmt.so; raises when it is missing or stale (no
    fallback: a query the procedure cannot take is an error, not a guess)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                               "g.build()'`")
        got = HASH_PATH.read_text().strip() if HASH_PATH.exists() else "missing"
        if got != source_hash():
            raise RuntimeError(f"{LIB_PATH} was not built from the current sources: rebuild it")
        lib = ctypes.CDLL(str(LIB_PATH))
        for name, (res, argtypes) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, argtypes
        _lib = lib
        return lib


class Unsupported(ValueError):
    """A node the procedure has no encoding for."""


def _limbs(v: int, w: int) -> List[int]:
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range((w + 31) // 32)]


class _Table:
    """The post-order node table of a set of roots (shared subterms once)."""

    def __init__(self):
        self.index: Dict[int, int] = {}
        self.keep: List[Node] = []
        self.nodes: List[int] = []           # rows not yet sent (a session keeps the sent ones)
        self.args: List[int] = []
        self.limbs: List[int] = [0]
        self.sent = 0                        # nodes the session already holds
        self.vars: Dict[str, Tuple[int, int]] = {}          # name -> (id, width)
        self.arrays: Dict[str, Tuple[int, int, int]] = {}   # name -> (id, domain, range)
        self.funcs: Dict[str, Tuple[int, tuple, int]] = {}  # name -> (id, domain widths, range)

    def add(self, root: Node) -> int:
        stack = [(root, False)]
        while stack:
            n, ready = stack.pop()
            if id(n) in self.index:
                continue
            if not ready:
                stack.append((n, True))
                for a in reversed(n.args):
                    if id(a) not in self.index:
                        stack.append((a, False))
                continue
            self._emit(n)
        return self.index[id(root)]

    def _emit(self, n: Node) -> None:
        op = OPS.get(n.op)
        if op is None:
            raise Unsupported(f"no exact encoding for {n.op}")
        p0 = p1 = 0
        width = n.width
        if n.op == "const":
            p0 = len(self.limbs)
            self.limbs.extend(_limbs(n.param, n.width))
        elif n.op == "var":
            # z3 keys a constant by name and sort: x:4 and x:256 are two
            p0 = self.vars.setdefault((n.param, n.width), (len(self.vars), n.width))[0]
        elif n.op == "array":
            name, dom, rng = n.param
            p0 = self.arrays.setdefault((name, dom, rng), (len(self.arrays), dom, rng))[0]
            p1 = rng
        elif n.op in ("K", "store"):
            p1 = n.param[-1]
        elif n.op == "uf":
            name, dom, rng = n.param
            p0 = self.funcs.setdefault((name, tuple(dom), rng), (len(self.funcs), tuple(dom), rng))[0]
        elif n.op == "extract":
            p0, p1 = n.param
        elif n.op in ("zero_extend", "sign_extend"):
            p0 = n.param
        first = len(self.args)
        self.args.extend(self.index[id(a)] for a in n.args)
        self.index[id(n)] = len(self.keep)
        self.keep.append(n)
        self.nodes.extend((op, width, len(n.args), first, p0, p1))

    def take_new(self):
        """The rows added since the last call (arguments global, first_arg and
        constant limbs local to the returned arrays), and mark them sent."""
        out = (self.nodes, self.args, self.limbs)
        self.sent = len(self.keep)
        self.nodes, self.args, self.limbs = [], [], [0]
        return out


def _divides_by_application(conjuncts: Sequence[Node]) -> bool:
    """Whether a bvudiv / bvurem in the conjuncts divides by a function
    application (its divisor node, directly)."""
    return _any_node(conjuncts, lambda n: n.op in ("bvudiv", "bvurem") and len(n.args) == 2
                     and n.args[1].op == "uf")


def _multiplies_words(conjuncts: Sequence[Node]) -> bool:
    """Whether the conjuncts multiply two non-constant words of 64 bits or more
    (a product whose circuit only level-0 facts -- a bound on one factor --
    can fold)."""
    return _any_node(conjuncts, lambda n: (n.op == "bvmul" and n.width >= 64 or n.op == "bvumul_noovfl")
                     and len(n.args) == 2 and all(a.op != "const" for a in n.args))


def _any_node(conjuncts: Sequence[Node], pred) -> bool:
    seen, stack = set(), list(conjuncts)
    while stack:
        n = stack.pop()
        if id(n) in seen:
            continue
        seen.add(id(n))
        if pred(n):
            return True
        stack.extend(a for a in n.args if isinstance(a, Node))
    return False


class ExactSolver:
    """``check(conjuncts, minimize)`` -> ("sat", assignment) | ("unsat", None)
    | ("unknown", None), the assignment in the ModelRef form (name -> int,
    ArrayInterp, FuncInterp).  Budgets: conflicts and wall time per query.

    The queries of one analysis share most of their terms (the path's prefix,
    the keccak axioms, the calldata reads), so one session (ms_session_*) holds
    them all: a query sends only the nodes the session lacks and is decided
    under assumptions, over the clauses and lemmas its predecessors left.  The
    session restarts when its CNF passes `session_vars`."""

    def __init__(self, max_ms: int = 60000, max_conflicts: int = 50_000, minimize_ms: int = 60000,
                 session: bool = True, session_vars: int = 400_000, session_conflicts: int = 5_000):
        # the budget is a conflict count (deterministic: the same query order
        # gives the same verdicts on any host), with a wall-clock cap as a guard.
        # 50,000 conflicts take about 4 s on the GPU box's host cores, inside
        # the reference's default z3 timeout (support_args.py:12, 10 s); every
        # query the 18-contract field and BECToken -t 1 decide needs < 3,300
        # (profiles/r06/exact_budget.txt); the budget is spent by divisions
        # whose divisor is a Power() application (flag_array's packed bool
        # array: `word / 256**(i % 32)`, a 256-bit divider over a symbolic
        # divisor), a timeout that prunes, as the reference's does
        self.max_ms = max_ms
        self.max_conflicts = max_conflicts
        self.session_conflicts = session_conflicts
        self.minimize_ms = minimize_ms
        self.use_session = session
        self.session_vars = session_vars
        self._session = None
        self._table: Optional[_Table] = None
        self._lock = threading.Lock()
        self.stats: Dict[str, int] = {"calls": 0, "sat": 0, "unsat": 0, "unknown": 0, "ms": 0,
                                      "vars": 0, "clauses": 0, "conflicts": 0, "sessions": 0}

    def close(self) -> None:
        if self._session is not None:
            load().ms_session_close(self._session)
            self._session = None
            self._table = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, conjuncts: Sequence[Node], minimize: Sequence[Node] = (), max_ms: Optional[int] = None,
              fresh: bool = False):
        """The session first, on `session_conflicts`; a query it cannot decide
        within them is decided alone, on `max_conflicts`: its conjuncts asserted
        as units, whose level-0 consequences fold the gates (a bounded factor
        turns a 256 x 256 multiplier into a few rows) -- what the session's
        assumptions cannot do for a shared clause database.  `max_ms` caps the
        wall clock of each attempt."""
        cap = self.max_ms if max_ms is None else max_ms
        with self._lock:
            if not fresh and os.environ.get("MYTHSMT_MUL_FRESH", "1") != "0" and _multiplies_words(conjuncts):
                # a product of two words: decided alone, a bound on one factor is a
                # unit whose level-0 consequences fold the multiplier's rows (in a
                # session the bound is an assumption and the whole 256 x 256 array
                # is searched; BECToken -t 1 exact time 8.1 -> 6.5 s, the field's
                # 1.46 -> 1.24 s, same verdicts: profiles/r06/exact_budget.txt)
                self.stats["fresh_direct_mul"] = self.stats.get("fresh_direct_mul", 0) + 1
                fresh = True
            if not fresh and _divides_by_application(conjuncts):
                # a division by a function application (Power(256, i % 32)): decided
                # alone, its pinned points are units, and the blaster splits the
                # division into shifts (bvsat.cpp divisor_cases) -- in a session they
                # are assumptions, and every such query re-blasts a 512-bit divider
                self.stats["fresh_direct"] = self.stats.get("fresh_direct", 0) + 1
                fresh = True
            if not self.use_session or fresh or minimize:
                # the objectives are met bit by bit under assumptions: alone, the
                # query's units fold what the bounds fix (and no other query's
                # terms slow each of those solves)
                return self._check(conjuncts, minimize, cap, False, self.max_conflicts)
            st, a = self._check(conjuncts, minimize, cap, True, self.session_conflicts)
            if st != "unknown":
                return st, a
            self.stats["fresh_retries"] = self.stats.get("fresh_retries", 0) + 1
            self.stats["unknown"] -= 1
            self.stats["calls"] -= 1
            return self._check(conjuncts, minimize, cap, False, self.max_conflicts)

    def _check(self, conjuncts, minimize, max_ms, session: bool, max_conflicts: int):
        import numpy as np
        from .program import ArrayInterp, FuncInterp
        lib = load()
        if session and self._session is None:
            h = ctypes.c_void_p()
            if lib.ms_session_open(ctypes.byref(h)) != 0:
                raise RuntimeError("ms_session_open failed")
            self._session, self._table = h, _Table()
            self.stats["sessions"] += 1
        t = self._table if session else _Table()
        roots = [t.add(c) for c in conjuncts]
        mins = [t.add(m) for m in minimize]
        self.stats["calls"] += 1
        new_nodes, new_args, new_limbs = t.take_new()
        nodes = np.asarray(new_nodes or [0], dtype=np.uint32)
        args = np.asarray(new_args or [0], dtype=np.uint32)
        limbs = np.asarray(new_limbs, dtype=np.uint32)
        roots_a = np.asarray(roots or [0], dtype=np.uint32)
        mins_a = np.asarray(mins or [0], dtype=np.uint32)
        q = MsQuery(len(new_nodes) // 6, nodes.ctypes.data, args.ctypes.data, limbs.ctypes.data, len(roots),
                    roots_a.ctypes.data, len(mins), mins_a.ctypes.data, len(t.vars), len(t.arrays), len(t.funcs))
        lim = MsLimits(max_conflicts, max_ms, self.minimize_ms)
        dump = os.environ.get("MYTHSMT_DUMP")
        if dump and not session:        # diagnostics: the query as ms_solve sees it
            os.makedirs(dump, exist_ok=True)
            np.savez(os.path.join(dump, f"q{self.stats['calls']:05d}_{os.getpid()}.npz"), nodes=nodes, args=args,
                     limbs=limbs, roots=roots_a[:len(roots)], mins=mins_a[:len(mins)],
                     counts=np.asarray([len(t.vars), len(t.arrays), len(t.funcs)], dtype=np.uint32))
        st = MsStats()
        cap = 1 << 16
        while True:
            out = np.zeros(cap, dtype=np.uint32)
            n = ctypes.c_uint32(0)
            if session:
                rc = lib.ms_session_solve(self._session, ctypes.byref(q), ctypes.byref(lim), out.ctypes.data, cap,
                                          ctypes.byref(n), ctypes.byref(st))
                q.n_nodes = 0                    # appended: a retry sends nothing new
            else:
                rc = lib.ms_solve(ctypes.byref(q), ctypes.byref(lim), out.ctypes.data, cap, ctypes.byref(n),
                                  ctypes.byref(st))
            if rc != MS_ESPACE:
                break
            cap = int(n.value) + 16
        self.stats["ms"] += int(st.ms)
        self.stats["conflicts"] += int(st.conflicts)
        self.stats["vars"] = max(self.stats["vars"], int(st.vars))
        self.stats["clauses"] = max(self.stats["clauses"], int(st.clauses))
        if rc == MS_EINVAL:
            if session:
                self.close()
            raise Unsupported("ms_solve rejected the query")
        if session and int(st.vars) > self.session_vars:
            self.close()                          # the next query starts a fresh session
        if rc == MS_UNSAT:
            self.stats["unsat"] += 1
            return "unsat", None
        if rc == MS_UNKNOWN:
            self.stats["unknown"] += 1
            return "unknown", None
        self.stats["sat"] += 1
        words = out[: int(n.value)].tolist()
        pos = 0

        def take(w):
            nonlocal pos
            k = (w + 31) // 32
            v = 0
            for i in range(k):
                v |= int(words[pos + i]) << (32 * i)
            pos += k
            return v

        var_by_id = {v[0]: (k[0], v[1]) for k, v in t.vars.items()}
        arr_by_id = {v[0]: (k[0], v[1], v[2]) for k, v in t.arrays.items()}
        fn_by_id = {v[0]: (k[0], v[1], v[2]) for k, v in t.funcs.items()}
        assign: Dict[str, object] = {}
        while True:
            tag = words[pos]
            pos += 1
            if tag == 0:
                break
            ident = words[pos]
            pos += 1
            if tag == 3:
                name, w = var_by_id[ident]
                assign[name] = take(w)
            elif tag == 1:
                name, dom, rng = arr_by_id[ident]
                idx = take(dom)
                val = take(rng)
                interp = assign.setdefault(name, ArrayInterp(0, {}))
                interp.entries[idx] = val
            else:
                name, dom, rng = fn_by_id[ident]
                xs = tuple(take(w) for w in dom)
                val = take(rng)
                interp = assign.setdefault(name, FuncInterp(0, {}))
                interp.entries[xs] = val
        return "sat", assign
