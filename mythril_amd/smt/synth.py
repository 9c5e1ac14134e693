"""C4 — synthetic bit-vector constraint DAGs x candidate models.

"1,000,000 DAGs x 4,096 models, seed 0x5EED0004.  Each DAG is a spine of depth
32: each level applies one op to (spine, fresh leaf).  Op mix: add/sub 20 %,
and/or/xor/not 20 %, mul 8 %, shl/lshr/ashr 8 %, extract+zero-ext/concat 8 %,
ite 8 %, eq/ult/ugt/slt 20 % (compare nodes feed an ite or Bool And), udiv/urem
4 %; leaves = one of V=16 BV256 vars (70 %) or a constant (30 %: 0, 1, 2^k,
2^256-1, small ints).  Root = Bool.  Models: 50 % uniform, 25 % small (<2^16),
25 % special (0, 1, 2^255, 2^256-1, address-shaped)."

The mix sums to 96 %; it is renormalised.  Remaining free choices, fixed here:
`not` is bvnot(spine) (its leaf unused); shift amounts are constants in
[0, 256); extract+zero-ext keeps 128 bits at lo in {0, 64, 128}, concat joins the
low halves of spine and leaf; the `ite` class is ite(leaf <u spine, spine, leaf);
a compare feeding an ite is ite(cmp(spine, leaf), spine, leaf), one feeding a
Bool And is conjoined into the DAG's Bool accumulator; the root is
(spine >u leaf_root) AND accumulator.

Programs are emitted directly in the kernel-2 format with numpy (1M DAGs in a
few seconds); ``dag_expr`` rebuilds DAG i as an expression (expr.Node) from the
same draws so tests can evaluate it independently.
"""
from __future__ import annotations

import os

import numpy as np

from .expr import Node, const as cnode, var as vnode
from .program import (OPCODE, REF_ACC, REF_CONST, REF_SLOT, REF_VAR, ModelPool, ProgramBatch,
                      limbs)

C4_SEED = 0x5EED0004
N_VARS = 16
LEVELS = 32
# classes: addsub, logic, mul, shift, extcat, ite, cmp, divrem
P = np.array([0.20, 0.20, 0.08, 0.08, 0.08, 0.08, 0.20, 0.04])
P = P / P.sum()
ADDSUB, LOGIC, MUL, SHIFT, EXTCAT, ITE, CMP, DIVREM = range(8)

# constant pool: 0, 1, 2^256-1, 2^k (k < 256), small s (s < 2^16)
C_ZERO, C_ONE, C_ONES, C_POW, C_SMALL = 0, 1, 2, 3, 259
N_CONSTS = 259 + (1 << 16)
M256 = (1 << 256) - 1


def const_pool() -> np.ndarray:
    vals = [0, 1, M256] + [1 << k for k in range(256)]
    pool = np.zeros((N_CONSTS, 8), dtype=np.uint32)
    for i, v in enumerate(vals):
        pool[i] = limbs(v)
    s = np.arange(1 << 16, dtype=np.uint32)
    pool[C_SMALL:, 0] = s
    return pool


def const_value(idx: int) -> int:
    if idx == C_ZERO:
        return 0
    if idx == C_ONE:
        return 1
    if idx == C_ONES:
        return M256
    if idx < C_SMALL:
        return 1 << (idx - C_POW)
    return idx - C_SMALL


class Draws:
    """All random choices of a C4 batch."""

    def __init__(self, n: int, seed: int = C4_SEED):
        rng = np.random.Generator(np.random.PCG64(seed))
        L = LEVELS
        self.n = n
        self.cls = rng.choice(8, size=(n, L), p=P).astype(np.int8)
        self.sub = rng.integers(0, 12, size=(n, L), dtype=np.int8)      # sub-op selector
        self.use_and = rng.random((n, L)) < 0.5
        self.leaf_is_var = rng.random((n, L)) < 0.7
        self.leaf_var = rng.integers(0, N_VARS, (n, L), dtype=np.int64)
        ck = rng.integers(0, 5, (n, L))
        kexp = rng.integers(0, 256, (n, L))
        small = rng.integers(0, 1 << 16, (n, L))
        self.leaf_const = np.select([ck == 0, ck == 1, ck == 2, ck == 3],
                                    [C_ZERO, C_ONE, C_POW + kexp, C_ONES],
                                    C_SMALL + small).astype(np.int64)
        self.shift = rng.integers(0, 256, (n, L), dtype=np.int64)
        self.lo = rng.choice([0, 64, 128], size=(n, L))
        self.spine0 = rng.integers(0, N_VARS, n, dtype=np.int64)
        self.root_is_var = rng.random(n) < 0.7
        self.root_var = rng.integers(0, N_VARS, n, dtype=np.int64)
        self.root_const = C_SMALL + rng.integers(0, 1 << 16, n)

    def leaf_ref(self):
        return np.where(self.leaf_is_var, (REF_VAR << 30) | self.leaf_var,
                        (REF_CONST << 30) | self.leaf_const).astype(np.uint32)


def _w0(op, width, store_slot=None):
    w = np.uint32(OPCODE[op] | (width << 8))
    return w


def c4_programs(dr: Draws) -> ProgramBatch:
    """Kernel-2 programs of every DAG, built with array operations, in the form
    flatten.Compiler emits for dag_expr(dr, i) (copy-free operand references,
    select-of-compare folded to min/max by flatten._fold_select, zero-extension
    of a computed value aliased) with this generator's own slot schedule, which
    never needs more than two slots: S0 keeps the spine across a compare that
    feeds the Bool accumulator, S1 the accumulator.

    The spine of level l is an operand reference `spin`: ACC when the previous
    level's last instruction left it in the accumulator, S0 when a compare-And
    level sat in between, or a leaf (the head variable, or the leaf an
    ite(spine == leaf, spine, leaf) level reduces to)."""
    n, L = dr.n, LEVELS
    cap = 3 * L + 2
    out = np.zeros((n, cap, 4), dtype=np.uint32)
    cnt = np.zeros(n, dtype=np.int64)
    last = np.full(n, -1, dtype=np.int64)
    rows_all = np.arange(n)
    leaf = dr.leaf_ref()
    ACC = np.uint32(REF_ACC << 30)
    S0 = np.uint32(REF_SLOT << 30 | 0)
    S1 = np.uint32(REF_SLOT << 30 | 1)

    def emit(mask, w0, a, b=0, c=0):
        r = rows_all[mask]
        if r.size == 0:
            return
        k = cnt[r]

        def pick(x):
            return x if np.ndim(x) == 0 else np.asarray(x)[mask]
        out[r, k, 0] = pick(w0)
        out[r, k, 1] = pick(a)
        out[r, k, 2] = pick(b)
        out[r, k, 3] = pick(c)
        last[r] = k
        cnt[r] += 1

    def w(op, width):
        return np.uint32(OPCODE[op] | (width << 8)) if isinstance(op, str) else \
            (np.asarray(op, dtype=np.uint32) | np.uint32(width << 8))

    # liveness (the compiler only emits what the root reaches): a level's spine
    # is dead when every path to the root passes an ite(spine == leaf, ..)
    # level before a compare uses it; a dead level emits nothing
    live = np.zeros((n, L), dtype=bool)
    nxt = np.ones(n, dtype=bool)
    for l in range(L - 1, -1, -1):
        c = dr.cls[:, l]
        is_and = (c == CMP) & dr.use_and[:, l]
        is_eq = (c == CMP) & ~dr.use_and[:, l] & (dr.sub[:, l] % 4 == 0)
        live[:, l] = ~is_eq & (is_and | nxt)
        nxt = np.where(is_eq, False, np.where(is_and, True, nxt))
    spin = ((REF_VAR << 30) | dr.spine0).astype(np.uint32)    # the head variable, no copy
    spin_acc = np.zeros(n, dtype=bool)
    n_and = np.zeros(n, dtype=np.int64)
    for l in range(L):
        cls, sub, lf = dr.cls[:, l], dr.sub[:, l].astype(np.int64), leaf[:, l]
        cls = np.where(live[:, l] | (cls == CMP), cls, -1)          # dead levels: nothing
        A = np.where(spin_acc, ACC, spin).astype(np.uint32)
        m_cmp = cls == CMP
        m_and = m_cmp & dr.use_and[:, l]
        # a compare-And level keeps the spine: save it to S0 if it is in the accumulator
        sv = m_and & spin_acc
        out[rows_all[sv], last[sv], 0] |= np.uint32(1 << 17)          # store to slot 0
        produced = np.zeros(n, dtype=bool)
        m = cls == ADDSUB
        emit(m, w(np.where(sub % 2 == 0, OPCODE["bvadd"], OPCODE["bvsub"]), 256), A, lf)
        produced |= m
        m = cls == LOGIC
        lop = np.choose(sub % 4, [OPCODE["bvand"], OPCODE["bvor"], OPCODE["bvxor"], OPCODE["bvnot"]])
        emit(m, w(lop, 256), A, np.where(sub % 4 == 3, 0, lf).astype(np.uint32))
        produced |= m
        m = cls == MUL
        emit(m, w("bvmul", 256), A, lf)
        produced |= m
        m = cls == SHIFT
        sop = np.choose(sub % 3, [OPCODE["bvshl"], OPCODE["bvlshr"], OPCODE["bvashr"]])
        emit(m, w(sop, 256), A, ((REF_CONST << 30) | (C_SMALL + dr.shift[:, l])).astype(np.uint32))
        produced |= m
        m = (cls == EXTCAT) & (sub % 2 == 0)          # zero_extend(extract): the extract alone
        emit(m, w("extract", 128), A, dr.lo[:, l].astype(np.uint32))
        produced |= m
        m = (cls == EXTCAT) & (sub % 2 == 1)          # concat(low128(spine), low128(leaf))
        emit(m, np.uint32(OPCODE["extract"] | (128 << 8) | (1 << 17)), A, 0)     # -> S0
        emit(m, w("extract", 128), lf, 0)
        if _LEGACY_CONCAT:                            # A/B runs against builds before rconcat
            emit(m, w("concat", 256), S0, ACC, 128)
        else:
            emit(m, w("rconcat", 256), ACC, S0, 128)  # concat(S0, acc): the accumulator stays operand A
        produced |= m
        m = cls == ITE                                # ite(leaf <u spine, spine, leaf)
        emit(m, w("bvumax", 256), A, lf)
        produced |= m
        m_sel = m_cmp & ~dr.use_and[:, l]             # ite(cmp(spine, leaf), spine, leaf)
        cop = sub % 4                                 # eq, ult, ugt, slt
        fold = np.choose(cop, [0, OPCODE["bvumin"], OPCODE["bvumax"], OPCODE["bvsmin"]])
        m = m_sel & (cop != 0) & live[:, l]
        emit(m, w(fold, 256), A, lf)
        produced |= m
        m_eq = m_sel & (cop == 0)                     # = leaf: no instruction
        m = cls == DIVREM
        emit(m, w(np.where(sub % 2 == 0, OPCODE["bvudiv"], OPCODE["bvurem"]), 256), A, lf)
        produced |= m
        # compare feeding the Bool accumulator (slot 1)
        cmpop = np.choose(cop, [OPCODE["eq"], OPCODE["bvult"], OPCODE["bvugt"], OPCODE["bvslt"]])
        first = m_and & (n_and == 0)
        later = m_and & (n_and > 0)
        emit(first, np.asarray(cmpop, dtype=np.uint32) | np.uint32((1 << 8) | (1 << 17) | (1 << 18)),
             A, lf, 256)
        emit(later, w(cmpop, 1), A, lf, 256)
        emit(later, np.uint32(OPCODE["and"] | (1 << 8) | (1 << 17) | (1 << 18)), ACC, S1)
        n_and += m_and
        # the next level's spine
        spin = np.where(m_and, np.where(spin_acc, S0, spin), spin)
        spin = np.where(m_eq, lf, spin).astype(np.uint32)
        spin_acc = np.where(produced, True, np.where(m_and | m_eq, False, spin_acc))
        spin = np.where(produced, ACC, spin).astype(np.uint32)
    # root: (spine >u leaf_root) [and accumulator]
    root_ref = np.where(dr.root_is_var, (REF_VAR << 30) | dr.root_var,
                        (REF_CONST << 30) | dr.root_const).astype(np.uint32)
    A = np.where(spin_acc, ACC, spin).astype(np.uint32)
    emit(np.ones(n, dtype=bool), w("bvugt", 1), A, root_ref, 256)
    emit(n_and > 0, w("and", 1), ACC, S1)
    valid = np.arange(cap)[None, :] < cnt[:, None]
    insns = out[valid]
    off = np.zeros(n + 1, dtype=np.uint32)
    off[1:] = np.cumsum(cnt)
    return ProgramBatch(insns.astype(np.uint32), off, const_pool(), 2,
                        [f"x{i}" for i in range(N_VARS)], [256] * N_VARS)


def c4_models(n_models: int = 4096, seed: int = C4_SEED + 1) -> ModelPool:
    rng = np.random.Generator(np.random.PCG64(seed))
    V = N_VARS
    vals = rng.integers(0, 1 << 32, (V, n_models, 8), dtype=np.uint64).astype(np.uint32)
    kind = rng.random((V, n_models))
    small = kind >= 0.5
    vals[small & (kind < 0.75), 1:] = 0
    vals[small & (kind < 0.75), 0] &= 0xFFFF
    spec = kind >= 0.75
    which = rng.integers(0, 5, (V, n_models))
    sv = np.zeros((5, 8), dtype=np.uint32)
    sv[1, 0] = 1
    sv[2, 7] = 0x80000000
    sv[3, :] = 0xFFFFFFFF
    for k in range(4):
        m = spec & (which == k)
        vals[m] = sv[k]
    m = spec & (which == 4)                                # address-shaped: 160 random bits
    vals[m, 5:] = 0
    return ModelPool(vals)


CHUNK = 1 << 17


def c4_chunks(n_dags: int):
    """C4 DAG index space in chunks of CHUNK; chunk k is Draws(.., C4_SEED + k)."""
    return [(k, k * CHUNK, min(CHUNK, n_dags - k * CHUNK)) for k in range((n_dags + CHUNK - 1) // CHUNK)]


def concat_programs(parts):
    insns = np.concatenate([p.insns for p in parts])
    offs = [np.zeros(1, dtype=np.uint64)]
    base = 0
    for p in parts:
        offs.append(p.prog_off[1:].astype(np.uint64) + base)
        base += int(p.prog_off[-1])
    off = np.concatenate(offs).astype(np.uint32)
    first = parts[0]
    return ProgramBatch(insns, off, first.consts, first.n_slots, first.var_names, first.var_widths)


def c4_batch(n_dags: int = 1_000_000, n_models: int = 4096, seed: int = C4_SEED,
             chunks=None):
    """Programs of the C4 DAGs (all chunks, or the listed chunk indices) + the model pool."""
    sel = c4_chunks(n_dags) if chunks is None else [c for c in c4_chunks(n_dags) if c[0] in set(chunks)]
    parts = [c4_programs(Draws(cnt, seed + k)) for k, _, cnt in sel]
    return concat_programs(parts), c4_models(n_models, seed + 0x1000)


# ---------------------------------------------------------------- expression form
def dag_expr(dr: Draws, i: int) -> Node:
    """DAG i of the batch as an expression, from the same draws (for tests)."""
    def leaf(l):
        if dr.leaf_is_var[i, l]:
            return vnode(f"x{dr.leaf_var[i, l]}", 256)
        return cnode(const_value(int(dr.leaf_const[i, l])), 256)

    spine = vnode(f"x{dr.spine0[i]}", 256)
    acc = None
    for l in range(LEVELS):
        c, s = int(dr.cls[i, l]), int(dr.sub[i, l])
        lf = leaf(l)
        if c == ADDSUB:
            spine = Node("bvadd" if s % 2 == 0 else "bvsub", 256, (spine, lf))
        elif c == LOGIC:
            spine = Node("bvnot", 256, (spine,)) if s % 4 == 3 else \
                Node(["bvand", "bvor", "bvxor"][s % 4], 256, (spine, lf))
        elif c == MUL:
            spine = Node("bvmul", 256, (spine, lf))
        elif c == SHIFT:
            spine = Node(["bvshl", "bvlshr", "bvashr"][s % 3], 256,
                         (spine, cnode(int(dr.shift[i, l]), 256)))
        elif c == EXTCAT:
            if s % 2 == 0:
                lo = int(dr.lo[i, l])
                spine = Node("zero_extend", 256, (Node("extract", 128, (spine,), (lo + 127, lo)),), 128)
            else:
                spine = Node("concat", 256, (Node("extract", 128, (spine,), (127, 0)),
                                             Node("extract", 128, (lf,), (127, 0))))
        elif c == ITE:
            spine = Node("ite", 256, (Node("bvult", 1, (lf, spine)), spine, lf))
        elif c == CMP:
            cmp = Node(["eq", "bvult", "bvugt", "bvslt"][s % 4], 1, (spine, lf))
            if dr.use_and[i, l]:
                acc = cmp if acc is None else Node("and", 1, (cmp, acc))
            else:
                spine = Node("ite", 256, (cmp, spine, lf))
        elif c == DIVREM:
            spine = Node("bvudiv" if s % 2 == 0 else "bvurem", 256, (spine, lf))
    rl = vnode(f"x{dr.root_var[i]}", 256) if dr.root_is_var[i] else \
        cnode(const_value(int(dr.root_const[i])), 256)
    root = Node("bvugt", 1, (spine, rl))
    return root if acc is None else Node("and", 1, (root, acc))


def model_dict(pool: ModelPool, m: int) -> dict:
    return {f"x{v}": int.from_bytes(pool.values[v, m].astype("<u4").tobytes(), "little")
            for v in range(pool.n_vars)}


# ---------------------------------------------------------------- algorithmic cost
# SURVEY §8(d) cost table per instruction (int32 ops at w = ceil(width/32) limbs)
# MYTH_C4_LEGACY_CONCAT=1 (scripts/ab_k2.py `lib:legacy`): emit concat(S0, acc),
# the form library builds before the accumulator-in-A rule accept
_LEGACY_CONCAT = os.environ.get("MYTH_C4_LEGACY_CONCAT") == "1"


def _insn_cost(op: int, width: int) -> float:
    w = max(1, (width + 31) // 32)
    name = [k for k, v in OPCODE.items() if v == op][0]
    if name in ("bvand", "bvor", "bvxor", "bvnot", "ite", "extract", "concat", "rconcat", "zero_extend",
                "sign_extend", "copy"):
        return float(w)
    if name in ("bvadd", "bvsub", "bvrsub", "bvneg"):
        return 2.0 * w
    if name in ("bvshl", "bvlshr", "bvashr", "bvumin", "bvumax", "bvsmin", "bvsmax"):
        return 3.0 * w          # min/max: the folded compare (2w) + select (w)
    if name == "bvmul":
        return w * (w + 1) / 2 + w * (w - 1) / 2 + 2.0 * w * w
    if name in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"):
        return 32.0 * w * w
    if name in ("and", "or", "not", "xor", "implies"):
        return 1.0
    return 2.0 * 8   # compares / overflow predicates on 256-bit operands


_DIVS = ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")


def division_count(batch: ProgramBatch) -> int:
    """Division / remainder instructions over all DAGs (one per eval each)."""
    ops = (batch.insns[:, 0] & 0xFF).astype(np.int64)
    return int(np.isin(ops, [OPCODE[n] for n in _DIVS if n in OPCODE]).sum())


def program_cost(batch: ProgramBatch, div_cost=None):
    """(int32 ops per constraint-eval summed over all DAGs, model bytes gathered per eval).
    div_cost replaces the §8(d) 32 w^2 charge of each division when given."""
    ops = (batch.insns[:, 0] & 0xFF).astype(np.int64)
    widths = ((batch.insns[:, 0] >> 8) & 0x1FF).astype(np.int64)
    table = {}
    total = 0.0
    key = ops * 512 + widths
    uniq, counts = np.unique(key, return_counts=True)
    divs = {OPCODE[n] for n in _DIVS if n in OPCODE}
    for k, c in zip(uniq, counts):
        op = int(k // 512)
        total += c * (div_cost if (div_cost is not None and op in divs) else _insn_cost(op, int(k % 512)))
    refs = batch.insns[:, 1:4]
    var_refs = int(((refs >> 30) == REF_VAR).sum())
    return total, 32.0 * var_refs
