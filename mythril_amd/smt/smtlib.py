"""SMT-LIB 2 for the SMT fallback: the query log of ``--solver-log`` and the
input of any external solver process.

The reference writes every query it sends to z3's Optimize as
``{solver_log}/{abs(hash(query))}.smt2`` holding ``Optimize.sexpr()``
(support/model.py:62-73).  z3 is not installed here, so the text is this
core's own SMT-LIB 2 rendering of the same query (declarations, one
``assert`` per constraint, ``minimize``/``maximize`` objectives,
``check-sat``/``get-model``) — semantically the query z3 receives, not z3's
byte-for-byte printout (parity unpinned; the file name uses a stable hash of
the rendered text instead of Python's per-process ``hash``).

``solver_process_backend(argv)`` turns any SMT-LIB 2 solver binary (z3 -in,
cvc5, bitwuzla …) into a ``solver.set_solver_backend`` callable: it feeds the
rendered query on stdin and reads ``sat``/``unsat``/``unknown`` and the model's
bit-vector and Bool constants.  None of those binaries exists in this image or
on the GPU box; the plumbing is tested with a stand-in process.
"""
from __future__ import annotations

import hashlib
import re
import subprocess
from pathlib import Path
from typing import Dict, Iterable, List, Sequence, Tuple

from .expr import Bool, Node

_BV_OPS = {"bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvand",
           "bvor", "bvxor", "bvshl", "bvlshr", "bvashr", "bvult", "bvule", "bvugt", "bvuge",
           "bvslt", "bvsle", "bvsgt", "bvsge", "bvnot", "bvneg", "concat"}
_BOOL_OPS = {"and", "or", "not", "xor", "=>"}


def _sort(width: int) -> str:
    return "Bool" if width == 1 else f"(_ BitVec {width})"


class _Printer:
    def __init__(self):
        self.decls: Dict[str, str] = {}
        self.lets: List[Tuple[str, str]] = []
        self.memo: Dict[Node, str] = {}

    def _decl(self, name: str, text: str):
        self.decls.setdefault(name, text)

    @staticmethod
    def _sym(name: str) -> str:
        return name if re.fullmatch(r"[A-Za-z_~!@$%^&*+=<>.?/-][A-Za-z0-9_~!@$%^&*+=<>.?/-]*", name) \
            else "|" + name.replace("|", "_") + "|"

    def term(self, root: Node) -> str:
        stack = [(root, False)]
        while stack:
            n, ready = stack.pop()
            if n in self.memo:
                continue
            if not ready:
                stack.append((n, True))
                stack.extend((c, False) for c in n.args if c not in self.memo)
                continue
            self.memo[n] = self._one(n, [self.memo[c] for c in n.args])
        return self.memo[root]

    def _one(self, n: Node, a: List[str]) -> str:
        op = n.op
        if op == "const":
            if n.width == 1:
                return "true" if n.param else "false"
            return f"(_ bv{n.param} {n.width})"
        if op == "var":
            s = self._sym(n.param)
            self._decl(n.param, f"(declare-fun {s} () {_sort(n.width)})")
            return s
        if op == "array":
            name, dom, rng = n.param
            s = self._sym(name)
            self._decl(name, f"(declare-fun {s} () (Array (_ BitVec {dom}) (_ BitVec {rng})))")
            return s
        if op == "K":
            dom, rng = n.param
            return f"((as const (Array (_ BitVec {dom}) (_ BitVec {rng}))) {a[0]})"
        if op == "store":
            return f"(store {a[0]} {a[1]} {a[2]})"
        if op == "select":
            return f"(select {a[0]} {a[1]})"
        if op == "uf":
            name, dom, rng = n.param
            s = self._sym(name)
            self._decl(name, f"(declare-fun {s} ({' '.join(_sort(w) for w in dom)}) {_sort(rng)})")
            return f"({s} {' '.join(a)})"
        if op == "ite":
            return f"(ite {a[0]} {a[1]} {a[2]})"
        if op == "extract":
            hi, lo = n.param
            return f"((_ extract {hi} {lo}) {a[0]})"
        if op in ("zero_extend", "sign_extend"):
            return f"((_ {op} {n.param}) {a[0]})"
        if op == "eq":
            return f"(= {a[0]} {a[1]})"
        if op == "distinct":
            return f"(distinct {a[0]} {a[1]})"
        if op == "implies":
            return f"(=> {a[0]} {a[1]})"
        if op in _BV_OPS or op in _BOOL_OPS:
            return f"({op} {' '.join(a)})"
        w = n.args[0].width
        if op == "bvadd_noovfl_u":      # top bit of the (w+1)-bit sum is 0
            return (f"(= ((_ extract {w} {w}) (bvadd ((_ zero_extend 1) {a[0]}) "
                    f"((_ zero_extend 1) {a[1]}))) #b0)")
        if op == "bvumul_noovfl":       # high w bits of the 2w-bit product are 0
            return (f"(= ((_ extract {2 * w - 1} {w}) (bvmul ((_ zero_extend {w}) {a[0]}) "
                    f"((_ zero_extend {w}) {a[1]}))) (_ bv0 {w}))")
        if op == "bvsub_noudfl_u":
            return f"(bvule {a[1]} {a[0]})"
        raise ValueError(f"no SMT-LIB rendering for {op}")


def to_smt2(constraints: Iterable, minimize: Sequence = (), maximize: Sequence = ()) -> str:
    """The query get_model hands its backend, as one SMT-LIB 2 script."""
    p = _Printer()
    body = []
    for c in constraints:
        raw = c.raw if hasattr(c, "raw") else c
        body.append(f"(assert {p.term(raw)})")
    for e in minimize:
        body.append(f"(minimize {p.term(e.raw if hasattr(e, 'raw') else e)})")
    for e in maximize:
        body.append(f"(maximize {p.term(e.raw if hasattr(e, 'raw') else e)})")
    return "\n".join(list(p.decls.values()) + body + ["(check-sat)", "(get-model)"]) + "\n"


def log_query(directory: str, text: str) -> Path:
    """support/model.py:62-73: one .smt2 file per backend query."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    f = d / f"{int(hashlib.sha256(text.encode()).hexdigest()[:15], 16)}.smt2"
    f.write_text(text)
    return f


_DEFINE = re.compile(r"\(define-fun\s+(\|[^|]*\||\S+)\s+\(\)\s+(Bool|\(_ BitVec (\d+)\))\s+"
                     r"(true|false|#x[0-9a-fA-F]+|#b[01]+|\(_ bv(\d+) \d+\))\s*\)")


def parse_model(text: str) -> Dict[str, int]:
    """The bit-vector / Bool constants of a (get-model) answer."""
    out: Dict[str, int] = {}
    for m in _DEFINE.finditer(text):
        name = m.group(1).strip("|")
        v = m.group(4)
        if v in ("true", "false"):
            out[name] = int(v == "true")
        elif v.startswith("#x"):
            out[name] = int(v[2:], 16)
        elif v.startswith("#b"):
            out[name] = int(v[2:], 2)
        else:
            out[name] = int(m.group(5))
    return out


def solver_process_backend(argv: Sequence[str]):
    """A set_solver_backend callable running an SMT-LIB 2 solver process."""
    from .solver import Model, ModelRef, SolverTimeOutException, UnsatError

    def backend(constraints, minimize, maximize, timeout_ms):
        text = to_smt2(constraints, minimize, maximize)
        try:
            r = subprocess.run(list(argv), input=text, capture_output=True, text=True,
                               timeout=max(timeout_ms, 1) / 1000.0)
        except subprocess.TimeoutExpired:
            raise SolverTimeOutException
        first = r.stdout.strip().split("\n", 1)[0].strip() if r.stdout else "unknown"
        if first == "unsat":
            raise UnsatError
        if first != "sat":
            raise SolverTimeOutException
        return Model([ModelRef(parse_model(r.stdout))])

    return backend
