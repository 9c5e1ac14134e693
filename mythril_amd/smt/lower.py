"""Lower array, uninterpreted-function and wide (257..512-bit) expressions to
the 256-bit operations kernel 2 evaluates.

* ``Select(Store(...Store(base, i1, v1)..., in, vn), j)`` (array.py:14-86) becomes
  ``ite(j == in, vn, ... ite(j == i1, v1, base[j]))`` — the last store with an
  equal index wins, as in SMT-LIB; ``base[j]`` is the K array's default or a
  table lookup of the model's interpretation of the symbolic array;
* ``f(x)`` (function.py:7-29; keccak256_N and its inverse, Power) becomes a table
  lookup of the model's function interpretation, keyed by up to 512 argument
  bits (two 256-bit chunks: one argument of <= 512 bits, or two <= 256-bit
  arguments);
* values wider than 256 bits (keccak inputs of 64 bytes, the 512-bit inverse)
  are split into 256-bit chunks through concat / extract / zero_extend /
  constants / ite / table parts, and ``==`` / ``!=`` on them into chunk-wise
  conjunctions.  Anything wider than 512 bits or other arithmetic on wide
  values stays on z3 (Unsupported).

The table op is ``Node("tab", width, (k0, k1), (table, part, lo))``: bits
[256*part + lo, 256*part + lo + width) of the interpretation's value at key
(k0, k1); k1 is the constant 0 for keys of at most 256 bits.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

from .expr import Node, const, var

WMAX = 256
KEY_MAX = 512


class Unsupported(Exception):
    pass


SELECT_SEP = "\x1f"       # never part of a variable name the expression layer makes


def select_var(array_name: str, index: int) -> str:
    """The model-pool variable standing for ``select(Array(array_name), index)``."""
    return f"{array_name}{SELECT_SEP}{index}"


def rng_ok(a: Node) -> bool:
    return a.param[2] <= WMAX


class TableSig:
    """What a table stands for: a symbolic array or an uninterpreted function."""
    __slots__ = ("name", "kind", "domain", "range")

    def __init__(self, name, kind, domain, rng):
        self.name, self.kind, self.domain, self.range = name, kind, tuple(domain), rng

    def key_chunks(self, args: Tuple[int, ...]) -> Tuple[int, int]:
        """(k0, k1) of an interpretation entry's argument values."""
        if len(args) == 1:
            x = args[0]
            return x & ((1 << 256) - 1), x >> 256
        return args[0], args[1]


class Lowering:
    def __init__(self):
        self.tables: Dict[str, TableSig] = {}
        self._memo: Dict[Node, Node] = {}
        self._slice_memo: Dict[tuple, Node] = {}

    # ---------------------------------------------------------- tables
    def _table(self, name, kind, domain, rng) -> str:
        sig = self.tables.get(name)
        if sig is None:
            self.tables[name] = TableSig(name, kind, domain, rng)
        elif sig.domain != tuple(domain) or sig.range != rng or sig.kind != kind:
            raise Unsupported(f"table {name} used with two signatures")
        return name

    def _tab(self, name: str, width: int, key: Tuple[Node, Node], part: int, lo: int = 0) -> Node:
        return Node("tab", width, key, (name, part, lo))

    def _key(self, args: Tuple[Node, ...]) -> Tuple[Node, Node]:
        if len(args) == 1:
            a = args[0]
            if a.width <= WMAX:
                return self.lower(a), const(0, 256)
            if a.width > KEY_MAX:
                raise Unsupported("table key wider than 512 bits")
            return self.slice(a, 0, 256), self.slice(a, 256, a.width)
        if len(args) == 2 and all(a.width <= WMAX for a in args):
            return self.lower(args[0]), self.lower(args[1])
        raise Unsupported("function arity / argument widths not supported on the device")

    # ---------------------------------------------------------- main pass
    def lower(self, n: Node) -> Node:
        """Equivalent DAG of <= 256-bit device ops (n itself at most 256 bits)."""
        if n.width > WMAX:
            raise Unsupported("wide value outside a comparison / key")
        hit = self._memo.get(n)
        if hit is not None:
            return hit
        out = self._lower(n)
        self._memo[n] = out
        return out

    def _lower(self, n: Node) -> Node:
        op = n.op
        if op in ("const", "var"):
            return n
        if op in ("eq", "distinct") and n.args[0].width > WMAX:
            a, b = n.args
            parts = []
            for lo in range(0, a.width, WMAX):
                hi = min(lo + WMAX, a.width)
                parts.append(Node("eq", 1, (self.slice(a, lo, hi), self.slice(b, lo, hi))))
            conj = parts[0] if len(parts) == 1 else Node("and", 1, tuple(parts))
            return conj if op == "eq" else Node("not", 1, (conj,))
        if op == "select":
            return self._select(n)
        if op == "uf":
            name, dom, rng = n.param
            self._table(name, "uf", dom, rng)
            return self._tab(name, n.width, self._key(n.args), 0)
        if any(a.width == 0 for a in n.args):
            raise Unsupported(f"array-sorted operand of {op}")
        if any(a.width > WMAX for a in n.args):
            if op == "extract":
                hi, lo = n.param
                return self.slice(n.args[0], lo, hi + 1)
            raise Unsupported(f"{op} on a value wider than 256 bits")
        args = tuple(self.lower(a) for a in n.args)
        if args == n.args:
            return n
        return Node(op, n.width, args, n.param)

    def _select(self, n: Node) -> Node:
        arr, idx = n.args
        if idx.width > WMAX:
            raise Unsupported("array index wider than 256 bits")
        j = self.lower(idx)
        stores: List[Tuple[Node, Node]] = []
        a = arr
        while a.op == "store":
            stores.append((a.args[1], a.args[2]))
            a = a.args[0]
        if a.op == "K":
            r = self.lower(a.args[0])
        elif a.op == "array" and j.op == "const" and rng_ok(a):
            # a constant index into a symbolic array (calldata bytes, a fixed
            # storage slot, an actor's balance) is one value per model: a model-pool
            # variable instead of a table lookup (no entry scan on the device, no
            # table rows on the host); program.select_var_value reads it back
            r = var(select_var(a.param[0], j.param), a.param[2])
        elif a.op == "array":
            name, dom, rng = a.param
            self._table(name, "array", (dom,), rng)
            r = self._tab(name, rng, (j, const(0, 256)), 0)
        else:
            raise Unsupported(f"array expression {a.op}")
        for i_k, v_k in reversed(stores):          # innermost first, outermost wins
            r = Node("ite", n.width, (Node("eq", 1, (j, self.lower(i_k))), self.lower(v_k), r))
        return r

    # ---------------------------------------------------------- wide values
    def slice(self, n: Node, lo: int, hi: int) -> Node:
        """<= 256-bit node for bits [lo, hi) of n (any width up to 512)."""
        if hi - lo > WMAX:
            raise Unsupported("slice wider than 256 bits")
        key = (n, lo, hi)
        hit = self._slice_memo.get(key)
        if hit is not None:
            return hit
        out = self._slice(n, lo, hi)
        self._slice_memo[key] = out
        return out

    def _slice(self, n: Node, lo: int, hi: int) -> Node:
        w = hi - lo
        if n.width <= WMAX:
            x = self.lower(n)
            if lo == 0 and hi == n.width:
                return x
            return Node("extract", w, (x,), (hi - 1, lo))
        op = n.op
        if op == "const":
            return const(n.param >> lo, w)
        if op == "concat":
            a, b = n.args
            wb = b.width
            if hi <= wb:
                return self.slice(b, lo, hi)
            if lo >= wb:
                return self.slice(a, lo - wb, hi - wb)
            return Node("concat", w, (self.slice(a, 0, hi - wb), self.slice(b, lo, wb)))
        if op == "zero_extend":
            a = n.args[0]
            wa = a.width
            if lo >= wa:
                return const(0, w)
            if hi <= wa:
                return self.slice(a, lo, hi)
            return Node("zero_extend", w, (self.slice(a, lo, wa),), hi - wa)
        if op == "extract":
            _, elo = n.param
            return self.slice(n.args[0], lo + elo, hi + elo)
        if op == "ite":
            c = self.lower(n.args[0])
            return Node("ite", w, (c, self.slice(n.args[1], lo, hi), self.slice(n.args[2], lo, hi)))
        if op in ("uf", "select"):
            if op == "uf":
                name, dom, rng = n.param
                self._table(name, "uf", dom, rng)
                key = self._key(n.args)
            else:
                arr, idx = n.args
                if arr.op != "array":
                    raise Unsupported("wide select over stores")
                name, dom, rng = arr.param
                self._table(name, "array", (dom,), rng)
                key = (self.lower(idx), const(0, 256))
            part, off = divmod(lo, WMAX)
            if off + w > WMAX:
                raise Unsupported("slice across a 256-bit table part")
            return self._tab(name, w, key, part, off)
        raise Unsupported(f"{op} on a value wider than 256 bits")
