"""Hash-consed bit-vector / Bool expression DAGs — the constraint format kernel 2 evaluates.

Mirrors the operator surface of mythril/laser/smt (bitvec.py:16-253,
bitvec_helper.py:30-246, bool.py:13-152) so that a LASER constraint list maps
node-for-node onto a program (flatten.py):

* ``BitVec.__lt__/__gt__/__le__/__ge__`` and ``/`` and ``>>`` are SIGNED
  (bitvec.py:140-190, 92-99, 221-231), exactly as in the reference;
* ``==`` / ``!=`` zero-pad the narrower side (``_padded_operation``, bitvec.py:16-22);
* ``ULE``/``UGE`` are ``Or(ULT, ==)`` / ``Or(UGT, ==)`` (bitvec_helper.py:85-105);
* overflow predicates follow z3's ``bvadd_noovfl``/``bvumul_noovfl`` and
  ``BVSubNoUnderflow`` (bitvec_helper.py:200-246).

Annotations (taint sets) are carried as frozensets and unioned the way
bitvec.py:63-136 does.  ``annotate`` adds to the set of *this* wrapper object in
place, as expression.py:37-43 does, so every holder of the object (a DUP'd stack
slot, an environment word) sees it; kernel 1's taint lanes carry the sets as
object handles + atom masks (mythril_amd/laser/taint.py).
"""
from __future__ import annotations

import weakref
from typing import Iterable, Optional, Tuple

# weak: a node lives while an expression (or a parent node) holds it, so the
# table does not grow with every concrete value the host layer materialises
_INTERN: "weakref.WeakValueDictionary[tuple, Node]" = weakref.WeakValueDictionary()


class Node:
    """Interned DAG node.  op: str; width: bits (1 for Bool); args: child nodes;
    param: const value / var name / (hi, lo) / extension count."""
    __slots__ = ("op", "width", "args", "param", "_hash", "__weakref__")

    def __new__(cls, op: str, width: int, args: Tuple["Node", ...] = (), param=None):
        key = (op, width, tuple(id(a) for a in args), param)
        n = _INTERN.get(key)
        if n is not None:
            return n
        n = object.__new__(cls)
        n.op, n.width, n.args, n.param = op, width, tuple(args), param
        n._hash = hash(key)
        _INTERN[key] = n
        return n

    def __hash__(self):
        return self._hash

    def __eq__(self, other):
        return self is other

    def __repr__(self):
        if self.op == "const":
            return f"{self.param:#x}:{self.width}"
        if self.op == "var":
            return f"{self.param}:{self.width}"
        return f"({self.op}{'' if self.param is None else ' ' + str(self.param)} " + \
               " ".join(map(repr, self.args)) + ")"


def mask(w: int) -> int:
    return (1 << w) - 1


def const(value: int, width: int) -> Node:
    return Node("const", width, (), value & mask(width))


def var(name: str, width: int) -> Node:
    return Node("var", width, (), name)


TRUE = const(1, 1)
FALSE = const(0, 1)


def _fold(op: str, width: int, args, param=None) -> Node:
    """Constant folding for all-constant arguments (what z3's simplify does to
    BitVecNumRef operands; keeps concrete values concrete), and x == x -> True."""
    if op in ("eq", "distinct") and len(args) == 2 and args[0] is args[1]:
        return TRUE if op == "eq" else FALSE
    if args and all(a.op == "const" for a in args):
        from .semantics import apply_op
        return const(apply_op(op, width, [a.param for a in args], [a.width for a in args], param),
                     width)
    return Node(op, width, tuple(args), param)


# --------------------------------------------------------------- wrappers
class Expression:
    __slots__ = ("raw", "annotations")

    def __init__(self, raw: Node, annotations: Optional[Iterable] = None):
        self.raw = raw
        self.annotations = frozenset(annotations or ())

    def size(self) -> int:
        return self.raw.width

    def annotate(self, annotation) -> None:
        """expression.py:37-43: add to this object's annotation set."""
        self.annotations = self.annotations | {annotation}

    def get_annotations(self, annotation_type):
        """expression.py:54-55."""
        return [a for a in self.annotations if isinstance(a, annotation_type)]

    @property
    def symbolic(self) -> bool:
        return self.raw.op != "const"

    @property
    def value(self):
        return None if self.symbolic else self.raw.param

    def __repr__(self):
        return repr(self.raw)


def _ann(*xs):
    out = frozenset()
    for x in xs:
        if isinstance(x, Expression):
            out = out | x.annotations
    return out


class Bool(Expression):
    @property
    def value(self):
        if self.raw.op == "const":
            return bool(self.raw.param)
        return None

    @property
    def is_true(self):
        return self.value is True

    @property
    def is_false(self):
        return self.value is False

    def __bool__(self):  # bool.py:72-80: unknown -> False
        return bool(self.value)

    def __eq__(self, other):  # type: ignore[override]
        o = other if isinstance(other, Bool) else Bool(const(int(bool(other)), 1))
        return Bool(_fold("eq", 1, (self.raw, o.raw)), _ann(self, other))

    def __ne__(self, other):  # type: ignore[override]
        return Not(self == other)

    def __hash__(self):
        return hash(self.raw)


def _bv(x, width=256) -> "BitVec":
    if isinstance(x, BitVec):
        return x
    if isinstance(x, Bool):
        return If(x, BitVec(const(1, 256)), BitVec(const(0, 256)))
    return BitVec(const(int(x), width))


def _pad(a: Node, b: Node):
    if a.width == b.width:
        return a, b
    if a.width < b.width:
        return Node("zero_extend", b.width, (a,), b.width - a.width) if a.op != "const" else \
            const(a.param, b.width), b
    return a, (Node("zero_extend", a.width, (b,), a.width - b.width) if b.op != "const" else
               const(b.param, a.width))


class BitVec(Expression):
    def _bin(self, op, other, signed_width=None):
        o = _bv(other, self.size())
        return BitVec(_fold(op, self.size(), (self.raw, o.raw)), _ann(self, o))

    def __add__(self, o): return self._bin("bvadd", o)
    def __radd__(self, o): return _bv(o, self.size())._bin("bvadd", self)
    def __sub__(self, o): return self._bin("bvsub", o)
    def __rsub__(self, o): return _bv(o, self.size())._bin("bvsub", self)
    def __mul__(self, o): return self._bin("bvmul", o)
    def __truediv__(self, o): return self._bin("bvsdiv", o)        # bitvec.py:92-99 signed
    def __and__(self, o): return self._bin("bvand", o)
    def __or__(self, o): return self._bin("bvor", o)
    def __xor__(self, o): return self._bin("bvxor", o)
    def __lshift__(self, o): return self._bin("bvshl", o)
    def __rshift__(self, o): return self._bin("bvashr", o)          # z3 >> is arithmetic

    def __invert__(self):
        return BitVec(_fold("bvnot", self.size(), (self.raw,)), self.annotations)

    def __neg__(self):
        return BitVec(_fold("bvneg", self.size(), (self.raw,)), self.annotations)

    def _cmp(self, op, other):
        o = _bv(other, self.size())
        return Bool(_fold(op, 1, (self.raw, o.raw)), _ann(self, o))

    # signed comparisons, as the reference's BitVec operators (bitvec.py:140-190)
    def __lt__(self, o): return self._cmp("bvslt", o)
    def __gt__(self, o): return self._cmp("bvsgt", o)
    def __le__(self, o): return self._cmp("bvsle", o)
    def __ge__(self, o): return self._cmp("bvsge", o)

    def __eq__(self, other):  # type: ignore[override]
        o = _bv(other, self.size())
        a, b = _pad(self.raw, o.raw)
        return Bool(_fold("eq", 1, (a, b)), _ann(self, other))

    def __ne__(self, other):  # type: ignore[override]
        o = _bv(other, self.size())
        a, b = _pad(self.raw, o.raw)
        return Bool(_fold("distinct", 1, (a, b)), _ann(self, other))

    def __hash__(self):
        return hash(self.raw)


# ---------------------------------------------------------- free functions
def _raw_bool(x) -> Node:
    if isinstance(x, Bool):
        return x.raw
    return TRUE if bool(x) else FALSE


def And(*args) -> Bool:
    raws = [_raw_bool(a) for a in args]
    if any(r is FALSE for r in raws):
        return Bool(FALSE, _ann(*args))
    raws = [r for r in raws if r is not TRUE]
    if not raws:
        return Bool(TRUE, _ann(*args))
    if len(raws) == 1:
        return Bool(raws[0], _ann(*args))
    return Bool(Node("and", 1, tuple(raws)), _ann(*args))


def Or(*args) -> Bool:
    raws = [_raw_bool(a) for a in args]
    if any(r is TRUE for r in raws):
        return Bool(TRUE, _ann(*args))
    raws = [r for r in raws if r is not FALSE]
    if not raws:
        return Bool(FALSE, _ann(*args))
    if len(raws) == 1:
        return Bool(raws[0], _ann(*args))
    return Bool(Node("or", 1, tuple(raws)), _ann(*args))


def Not(a) -> Bool:
    return Bool(_fold("not", 1, (_raw_bool(a),)), _ann(a))


def Xor(a, b) -> Bool:
    return Bool(_fold("xor", 1, (_raw_bool(a), _raw_bool(b))), _ann(a, b))


def Implies(a, b) -> Bool:
    return Bool(_fold("implies", 1, (_raw_bool(a), _raw_bool(b))), _ann(a, b))


def If(c, a, b) -> BitVec:
    cr = _raw_bool(c)
    a, b = _bv(a), _bv(b)
    if cr is TRUE:
        return BitVec(a.raw, _ann(c, a, b))
    if cr is FALSE:
        return BitVec(b.raw, _ann(c, a, b))
    return BitVec(Node("ite", a.size(), (cr, a.raw, b.raw)), _ann(c, a, b))


def _bvfn(op):
    def f(a, b):
        a, b = _bv(a), _bv(b, a.size() if isinstance(a, BitVec) else 256)
        return BitVec(_fold(op, a.size(), (a.raw, b.raw)), _ann(a, b))
    f.__name__ = op
    return f


UDiv, URem, SRem, LShR = _bvfn("bvudiv"), _bvfn("bvurem"), _bvfn("bvsrem"), _bvfn("bvlshr")
SDiv, SMod = _bvfn("bvsdiv"), _bvfn("bvsmod")


def _ucmp(op):
    def f(a, b):
        a = _bv(a)
        b = _bv(b, a.size())
        return Bool(_fold(op, 1, (a.raw, b.raw)), _ann(a, b))
    f.__name__ = op
    return f


ULT, UGT = _ucmp("bvult"), _ucmp("bvugt")


def ULE(a, b) -> Bool:  # bitvec_helper.py:85-95
    a = _bv(a)
    b = _bv(b, a.size())
    if a.raw.op == "const" and a.raw.param == 0:
        return Bool(TRUE, _ann(a, b))        # z3 simplify: 0 <=u x is true
    return Or(ULT(a, b), a == b)


def UGE(a, b) -> Bool:  # bitvec_helper.py:97-105
    a = _bv(a)
    b = _bv(b, a.size())
    if b.raw.op == "const" and b.raw.param == 0:
        return Bool(TRUE, _ann(a, b))        # z3 simplify: x >=u 0 is true (a zero-value transfer)
    return Or(UGT(a, b), a == b)


def Concat(*args) -> BitVec:
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = tuple(args[0])
    bvs = [_bv(a) for a in args]
    acc = bvs[0]
    for b in bvs[1:]:
        w = acc.size() + b.size()
        acc = BitVec(_fold("concat", w, (acc.raw, b.raw)), _ann(acc, b))
    return acc


def simplify_concat(parts) -> BitVec:
    """``simplify(Concat(parts))`` as the reference builds memory words and SHA3
    inputs (memory.py:56-82, instructions.py:1032-1039): z3's concat rewrites
    restated on the part sequence -- adjacent constants join into one constant,
    adjacent extracts of the same term over contiguous bit ranges join into one
    extract, and an extract of a term's full width is the term.  A part that is
    neither a constant nor an extract counts as the full-width extract of itself
    (parts are never taken apart).  The result depends only on the part
    sequence after these joins, so parts that were joined in advance (device
    runs, mythril_amd/laser/symbolic.py) give the same expression as the bytes
    they cover."""
    atoms: list = []              # ["c", value, width] | ["x", term, hi, lo]
    ann = frozenset()
    for p in parts:
        p = _bv(p, 8)
        ann = ann | p.annotations
        r = p.raw
        if r.op == "const":
            a = ["c", r.param, r.width]
        elif r.op == "extract":
            a = ["x", r.args[0], r.param[0], r.param[1]]
        else:
            a = ["x", r, r.width - 1, 0]
        if atoms:
            b = atoms[-1]
            if a[0] == "c" and b[0] == "c":
                b[1], b[2] = (b[1] << a[2]) | a[1], b[2] + a[2]
                continue
            if a[0] == "x" and b[0] == "x" and a[1] is b[1] and b[3] == a[2] + 1:
                b[3] = a[3]
                continue
        atoms.append(a)
    acc = None
    for a in atoms:
        if a[0] == "c":
            n = const(a[1], a[2])
        elif a[2] == a[1].width - 1 and a[3] == 0:
            n = a[1]
        else:
            n = _fold("extract", a[2] - a[3] + 1, (a[1],), (a[2], a[3]))
        acc = n if acc is None else _fold("concat", acc.width + n.width, (acc, n))
    return BitVec(acc, ann)


def Extract(hi: int, lo: int, a) -> BitVec:
    a = _bv(a)
    return BitVec(_fold("extract", hi - lo + 1, (a.raw,), (hi, lo)), a.annotations)


def ZeroExt(k: int, a) -> BitVec:
    a = _bv(a)
    return BitVec(_fold("zero_extend", a.size() + k, (a.raw,), k), a.annotations)


def SignExt(k: int, a) -> BitVec:
    a = _bv(a)
    return BitVec(_fold("sign_extend", a.size() + k, (a.raw,), k), a.annotations)


def BVAddNoOverflow(a, b, signed: bool) -> Bool:
    if signed:
        raise NotImplementedError("signed overflow predicates are evaluated by z3 on the host")
    a, b = _bv(a), _bv(b)
    return Bool(_fold("bvadd_noovfl_u", 1, (a.raw, b.raw)), _ann(a, b))


def BVMulNoOverflow(a, b, signed: bool) -> Bool:
    if signed:
        raise NotImplementedError("signed overflow predicates are evaluated by z3 on the host")
    a, b = _bv(a), _bv(b)
    return Bool(_fold("bvumul_noovfl", 1, (a.raw, b.raw)), _ann(a, b))


def BVSubNoUnderflow(a, b, signed: bool) -> Bool:
    if signed:
        raise NotImplementedError("signed overflow predicates are evaluated by z3 on the host")
    a, b = _bv(a), _bv(b)
    return Bool(_fold("bvsub_noudfl_u", 1, (a.raw, b.raw)), _ann(a, b))


class ConstWord(BitVec):
    """A concrete 256-bit word read back from a lane (LaserEVM._materialise):
    `BitVecVal(v, 256)` with its DAG node built on first use of `.raw`.  Most
    words a hook event materialises are only compared, read for `.value` or
    passed along, so the interning of a fresh constant is skipped for them."""
    __slots__ = ("_v", "_n")

    def __init__(self, v: int):
        self._v = v
        self._n = None
        self.annotations = _NO_ANN

    @property
    def raw(self) -> Node:
        n = self._n
        if n is None:
            n = self._n = const(self._v, 256)
        return n

    @raw.setter
    def raw(self, node: Node) -> None:            # unpickling / copy.copy
        self._n = node
        self._v = node.param

    @property
    def symbolic(self) -> bool:
        return False

    @property
    def value(self):
        return self._v

    def size(self) -> int:
        return 256


_NO_ANN = frozenset()


class _SymbolFactory:
    """mythril/laser/smt/__init__.py:37-154 symbol_factory surface."""

    @staticmethod
    def BitVecVal(value: int, size: int, annotations=None) -> BitVec:
        return BitVec(const(value, size), annotations)

    @staticmethod
    def BitVecSym(name: str, size: int, annotations=None) -> BitVec:
        return BitVec(var(name, size), annotations)

    @staticmethod
    def Bool(value: bool, annotations=None) -> Bool:
        return Bool(TRUE if value else FALSE, annotations)

    @staticmethod
    def BoolSym(name: str, annotations=None) -> Bool:
        return Bool(var(name, 1), annotations)


symbol_factory = _SymbolFactory()


# ----------------------------------------------------- arrays and functions
# Array-sorted nodes have width 0 and carry (domain, range) widths in `param`:
#   ("array", name, dom, rng)      symbolic array   (array.py:56-70 Array)
#   K:     args (default,)         constant array   (array.py:73-86 K)
#   store: args (array, index, value)
# select(array, index) and uf(args...) are bit-vector nodes of the range width.
def _select(arr: Node, idx: Node) -> Node:
    """Select with the rewrites z3's simplify applies (the reference reads
    storage as ``simplify(storage[item])``, account.py:75): walking the store
    chain from the newest store, a store at the same index term answers (the
    terms are hash-consed: identical means the same node), a store at a
    distinct constant index is skipped when the index is a constant too, and a
    constant array answers its default for any index; the first store neither
    rule decides stops the walk, and the select stays over the rest of the
    chain."""
    a = arr
    while True:
        if a.op == "store":
            key = a.args[1]
            if key is idx:
                return a.args[2]
            if idx.op == "const" and key.op == "const":
                a = a.args[0]
                continue
            break
        if a.op == "K":
            return a.args[0]
        break
    return Node("select", a.param[-1], (a, idx))


class BaseArray:
    """array.py:14-53: ``arr[k]`` is Select, ``arr[k] = v`` replaces raw by Store."""

    def __init__(self, raw: Node):
        self.raw = raw

    @property
    def domain(self) -> int:
        return self.raw.param[-2]

    @property
    def range(self) -> int:
        return self.raw.param[-1]

    def __getitem__(self, item) -> BitVec:
        if isinstance(item, slice):
            raise ValueError("Instance of BaseArray, does not support getitem with slices")
        k = _bv(item, self.domain)
        return BitVec(_select(self.raw, k.raw))          # array.py:21-28: no annotations

    def __setitem__(self, key, value) -> None:
        k = _bv(key, self.domain)
        v = _bv(value, self.range)
        self.raw = Node("store", 0, (self.raw, k.raw, v.raw), (self.domain, self.range))


class Array(BaseArray):
    def __init__(self, name: str, domain: int, value_range: int):
        super().__init__(Node("array", 0, (), (name, domain, value_range)))


class K(BaseArray):
    def __init__(self, domain: int, value_range: int, value: int):
        super().__init__(Node("K", 0, (const(value, value_range),), (domain, value_range)))


class Function:
    """function.py:7-29: an uninterpreted function over bit-vectors."""

    def __init__(self, name: str, domain, value_range: int):
        self.name = name
        self.domain = list(domain)
        self.range = value_range

    def __call__(self, *items) -> BitVec:
        args = tuple(_bv(x, w) for x, w in zip(items, self.domain))
        return BitVec(Node("uf", self.range, tuple(a.raw for a in args),
                           (self.name, tuple(self.domain), self.range)), _ann(*args))

