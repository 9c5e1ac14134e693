"""z3 / SMT-LIB bit-vector semantics on Python ints.

Used for constant folding while expressions are built (the job z3's simplify
does in the reference when every operand is a BitVecNumRef).  Division and
remainder by zero follow SMT-LIB: bvudiv x 0 = 2^w-1, bvurem x 0 = x,
bvsdiv x 0 = (x < 0 ? 1 : -1), bvsrem x 0 = x, bvsmod x 0 = x.
"""
from __future__ import annotations


def _m(w):
    return (1 << w) - 1


def _s(x, w):
    return x - (1 << w) if x >> (w - 1) & 1 else x


def _sdiv(a, b, w):
    if b == 0:
        return 1 if _s(a, w) < 0 else _m(w)
    sa, sb = _s(a, w), _s(b, w)
    q = abs(sa) // abs(sb)
    return (-q if (sa < 0) != (sb < 0) else q) & _m(w)


def _srem(a, b, w):
    if b == 0:
        return a
    sa, sb = _s(a, w), _s(b, w)
    r = abs(sa) % abs(sb)
    return (-r if sa < 0 else r) & _m(w)


def _smod(a, b, w):
    if b == 0:
        return a
    r = _srem(a, b, w)
    if r == 0 or (_s(r, w) < 0) == (_s(b, w) < 0):
        return r
    return (r + b) & _m(w)


def apply_op(op: str, width: int, vals, widths, param=None) -> int:
    """Value of `op` at result width `width` on operand values `vals` (operand
    widths `widths`)."""
    M = _m(width)
    a = vals[0] if vals else 0
    b = vals[1] if len(vals) > 1 else 0
    wa = widths[0] if widths else width
    if op == "bvadd":
        return (a + b) & M
    if op == "bvsub":
        return (a - b) & M
    if op == "bvmul":
        return (a * b) & M
    if op == "bvudiv":
        return M if b == 0 else a // b
    if op == "bvurem":
        return a if b == 0 else a % b
    if op == "bvsdiv":
        return _sdiv(a, b, width)
    if op == "bvsrem":
        return _srem(a, b, width)
    if op == "bvsmod":
        return _smod(a, b, width)
    if op == "bvand":
        return a & b
    if op == "bvor":
        return a | b
    if op == "bvxor":
        return a ^ b
    if op == "bvnot":
        return ~a & M
    if op == "bvneg":
        return -a & M
    if op == "bvshl":
        return (a << b) & M if b < width else 0
    if op == "bvlshr":
        return a >> b if b < width else 0
    if op == "bvashr":
        return (_s(a, width) >> min(b, width)) & M
    if op == "eq":
        return int(a == b)
    if op == "distinct":
        return int(a != b)
    if op == "bvult":
        return int(a < b)
    if op == "bvule":
        return int(a <= b)
    if op == "bvugt":
        return int(a > b)
    if op == "bvuge":
        return int(a >= b)
    if op == "bvslt":
        return int(_s(a, wa) < _s(b, wa))
    if op == "bvsle":
        return int(_s(a, wa) <= _s(b, wa))
    if op == "bvsgt":
        return int(_s(a, wa) > _s(b, wa))
    if op == "bvsge":
        return int(_s(a, wa) >= _s(b, wa))
    if op == "and":
        return int(all(v & 1 for v in vals))
    if op == "or":
        return int(any(v & 1 for v in vals))
    if op == "not":
        return (a & 1) ^ 1
    if op == "xor":
        return (a ^ b) & 1
    if op == "implies":
        return int(not (a & 1) or (b & 1))
    if op == "ite":
        return vals[1] if a & 1 else vals[2]
    if op == "concat":
        return ((a << widths[1]) | b) & M
    if op == "extract":
        hi, lo = param
        return (a >> lo) & M
    if op == "zero_extend":
        return a
    if op == "sign_extend":
        return (a | (_m(width) ^ _m(wa))) if a >> (wa - 1) & 1 else a
    if op == "bvadd_noovfl_u":
        return int(a + b <= _m(wa))
    if op == "bvumul_noovfl":
        return int(a * b <= _m(wa))
    if op == "bvsub_noudfl_u":
        return int(b <= a)
    raise ValueError(f"unknown op {op}")
