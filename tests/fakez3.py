"""Test-only stand-in for the z3 Python API surface mythril_amd.bridge.to_dag
walks (the reference's mypy-stubs/z3/__init__.pyi: ExprRef.decl/children/sort,
FuncDeclRef.kind/name/params, BitVecNumRef.as_long, SortRef.kind/size/domain/
range).  The Z3_OP_* / Z3_*_SORT constants are arbitrary distinct ints: the
converter looks kinds up by NAME in the module it is given, so real z3's
numbering never matters.  z3 itself is absent here: parity unpinned."""
import itertools

_OPS = ["BNUM", "TRUE", "FALSE", "UNINTERPRETED", "BADD", "BSUB", "BMUL", "BUDIV", "BUDIV_I",
        "BUREM", "BUREM_I", "BSDIV", "BSDIV_I", "BSREM", "BSREM_I", "BSMOD", "BSMOD_I", "BAND",
        "BOR", "BXOR", "BNOT", "BNEG", "BSHL", "BLSHR", "BASHR", "ULT", "UGT", "ULEQ", "UGEQ",
        "SLT", "SGT", "SLEQ", "SGEQ", "EQ", "DISTINCT", "AND", "OR", "NOT", "XOR", "IMPLIES",
        "ITE", "CONCAT", "EXTRACT", "ZERO_EXT", "SIGN_EXT", "SELECT", "STORE", "CONST_ARRAY",
        "BSMUL_NO_OVFL"]
for _k, _n in enumerate(_OPS):
    globals()["Z3_OP_" + _n] = 1000 + 7 * _k
Z3_BOOL_SORT, Z3_BV_SORT, Z3_ARRAY_SORT = 1, 4, 5
_ids = itertools.count(1)


class Sort:
    def __init__(self, kind, size=None, dom=None, rng=None):
        self._k, self._s, self._d, self._r = kind, size, dom, rng

    def kind(self):
        return self._k

    def size(self):
        return self._s

    def domain(self):
        return self._d

    def range(self):
        return self._r


def BoolSort():
    return Sort(Z3_BOOL_SORT)


def BitVecSort(w):
    return Sort(Z3_BV_SORT, w)


def ArraySort(d, r):
    return Sort(Z3_ARRAY_SORT, dom=d, rng=r)


class Decl:
    def __init__(self, kind, name, params=()):
        self._k, self._n, self._p = kind, name, list(params)

    def kind(self):
        return self._k

    def name(self):
        return self._n

    def params(self):
        return self._p


class Expr:
    def __init__(self, op, sort, args=(), name=None, params=(), value=None):
        self._d = Decl(globals()["Z3_OP_" + op], name or op.lower(), params)
        self._s, self._a, self._v = sort, list(args), value
        self._id = next(_ids)

    def decl(self):
        return self._d

    def children(self):
        return self._a

    def sort(self):
        return self._s

    def as_long(self):
        return self._v

    def get_id(self):
        return self._id

    def size(self):
        return self._s.size()


def BitVecVal(v, w):
    return Expr("BNUM", BitVecSort(w), value=v % (1 << w))


def BitVec(name, w):
    return Expr("UNINTERPRETED", BitVecSort(w), name=name)


def Bool(name):
    return Expr("UNINTERPRETED", BoolSort(), name=name)


def BoolVal(b):
    return Expr("TRUE" if b else "FALSE", BoolSort())


def Array(name, d, r):
    return Expr("UNINTERPRETED", ArraySort(BitVecSort(d), BitVecSort(r)), name=name)


def K(d, v):
    return Expr("CONST_ARRAY", ArraySort(BitVecSort(d), v.sort()), [v])


def Select(a, i):
    return Expr("SELECT", a.sort().range(), [a, i])


def Store(a, i, v):
    return Expr("STORE", a.sort(), [a, i, v])


def Function(name, dom_widths, rng):
    def app(*args):
        return Expr("UNINTERPRETED", BitVecSort(rng), args, name=name)
    return app


def bv(op, *args):
    return Expr(op, args[0].sort(), args)


def pred(op, *args):
    return Expr(op, BoolSort(), args)


def If(c, a, b):
    return Expr("ITE", a.sort(), [c, a, b])


def Concat(*args):
    return Expr("CONCAT", BitVecSort(sum(a.size() for a in args)), args)


def Extract(hi, lo, a):
    return Expr("EXTRACT", BitVecSort(hi - lo + 1), [a], params=(hi, lo))


def ZeroExt(k, a):
    return Expr("ZERO_EXT", BitVecSort(a.size() + k), [a], params=(k,))


def SignExt(k, a):
    return Expr("SIGN_EXT", BitVecSort(a.size() + k), [a], params=(k,))


# ---- the constructors mythril_amd.bridge.from_dag calls (z3py's names) ----------
def _bool(op, *args):
    return Expr(op, BoolSort(), args)


def _w(x):
    return x.sort().size()


def UDiv(a, b): return bv("BUDIV", a, b)
def URem(a, b): return bv("BUREM", a, b)
def SRem(a, b): return bv("BSREM", a, b)
def LShR(a, b): return bv("BLSHR", a, b)
def ULT(a, b): return _bool("ULT", a, b)
def UGT(a, b): return _bool("UGT", a, b)
def ULE(a, b): return _bool("ULEQ", a, b)
def UGE(a, b): return _bool("UGEQ", a, b)
def And(*a): return _bool("AND", *a)
def Or(*a): return _bool("OR", *a)
def Not(a): return _bool("NOT", a)
def Xor(a, b): return _bool("XOR", a, b)
def Implies(a, b): return _bool("IMPLIES", a, b)
def Distinct(a, b): return _bool("DISTINCT", a, b)


def _function(name, *sorts):
    rng = sorts[-1]
    if isinstance(rng, int):              # this fake's older form: (name, domain widths, range width)
        rng = BitVecSort(rng)

    def app(*args):
        return Expr("UNINTERPRETED", rng, args, name=name)
    return app


Function = _function          # z3py: Function(name, *domain_sorts, range_sort)


def Array(name, dom, rng):  # noqa: F811  (z3py: Array(name, domain_sort, range_sort))
    if isinstance(dom, int):
        dom, rng = BitVecSort(dom), BitVecSort(rng)
    return Expr("UNINTERPRETED", ArraySort(dom, rng), name=name)


def K(dom, v):  # noqa: F811
    if isinstance(dom, int):
        dom = BitVecSort(dom)
    return Expr("CONST_ARRAY", ArraySort(dom, v.sort()), [v])


def _op(name):
    def f(self, other):
        return bv(name, self, other)
    return f


def _cmp(name):
    def f(self, other):
        return _bool(name, self, other)
    return f


Expr.__add__ = _op("BADD")
Expr.__sub__ = _op("BSUB")
Expr.__mul__ = _op("BMUL")
Expr.__truediv__ = _op("BSDIV")
Expr.__mod__ = _op("BSMOD")
Expr.__and__ = _op("BAND")
Expr.__or__ = _op("BOR")
Expr.__xor__ = _op("BXOR")
Expr.__lshift__ = _op("BSHL")
Expr.__rshift__ = _op("BASHR")
Expr.__invert__ = lambda self: bv("BNOT", self)
Expr.__neg__ = lambda self: bv("BNEG", self)
Expr.__lt__ = _cmp("SLT")
Expr.__gt__ = _cmp("SGT")
Expr.__le__ = _cmp("SLEQ")
Expr.__ge__ = _cmp("SGEQ")
Expr.__eq__ = _cmp("EQ")
Expr.__ne__ = _cmp("DISTINCT")
Expr.__hash__ = lambda self: self._id
