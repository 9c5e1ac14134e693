"""Compile constraint sets (expression DAGs) into kernel-2 register programs.

``get_model`` hands quick-sat ``simplify(And(*constraints))`` (support/model.py:51-54);
here every constraint set becomes one straight-line program whose last
instruction leaves the conjunction's truth value in the accumulator:

1. the DAG's internal nodes are scheduled post-order, each shared node once
   (hash-consing = the reference's z3 AST sharing), larger operand subtrees
   first so the last-computed operand is still in the accumulator;
2. a node consumed only by the very next instruction travels in the
   accumulator; every other node is stored to a slot, slots are reused by a
   linear scan over live ranges (at most MAX_SLOTS);
3. leaves are operand references: variables index the model pool, constants a
   deduplicated pool.
Sets that need more slots or wider than 256-bit values raise Unsupported and
stay on z3 (the prefilter may only ever answer SAT).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from .expr import Bool, Node, TRUE
from .lower import Lowering, Unsupported
from .program import (MAX_SLOTS, OPCODE, REF_ACC, REF_CONST, REF_SLOT, REF_VAR, TAB_LO_SHIFT,
                      TAB_PART_SHIFT, TILE_INSNS, ProgramBatch, enc_w0, limbs, ref)

_MAP = {"and": "and", "or": "or", "not": "not", "xor": "xor", "implies": "implies"}
_CMP = {"eq", "distinct", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
        "bvadd_noovfl_u", "bvumul_noovfl", "bvsub_noudfl_u"}
# The accumulator is only ever operand A (bv_eval.cuh keeps A in the
# accumulator's registers).  A previous result needed as operand B is swapped
# into A for these ops (the op itself, or its operand-swapped form), otherwise
# it goes through a slot.
_COMMUTATIVE = {"bvadd", "bvmul", "bvand", "bvor", "bvxor", "eq", "distinct", "and", "or", "xor",
                "bvadd_noovfl_u", "bvumul_noovfl", "bvumin", "bvumax", "bvsmin", "bvsmax"}
_SWAPPED = {"bvult": "bvugt", "bvugt": "bvult", "bvule": "bvuge", "bvuge": "bvule",
            "bvslt": "bvsgt", "bvsgt": "bvslt", "bvsle": "bvsge", "bvsge": "bvsle",
            "bvsub": "bvrsub", "bvrsub": "bvsub", "concat": "rconcat", "rconcat": "concat"}


def _acc_ok(op: str, k: int) -> bool:
    """Can operand k of `op` be the accumulator (after a swap when k == 1)?"""
    return k == 0 or (k == 1 and (op in _COMMUTATIVE or op in _SWAPPED))


_MINMAX = {  # ite(cmp(x, y), x, y) -> op(x, y); ite(cmp(x, y), y, x) -> the other one
    "bvult": ("bvumin", "bvumax"), "bvule": ("bvumin", "bvumax"),
    "bvugt": ("bvumax", "bvumin"), "bvuge": ("bvumax", "bvumin"),
    "bvslt": ("bvsmin", "bvsmax"), "bvsle": ("bvsmin", "bvsmax"),
    "bvsgt": ("bvsmax", "bvsmin"), "bvsge": ("bvsmax", "bvsmin"),
}


def _fold_select(root: Node) -> Node:
    """Peephole over the lowered DAG: a select between the two operands of its
    own compare is one min/max instruction, and ite(x == y, x, y) is y (with
    x == y both branches are the same number).  Ties pick either operand: the
    value is the same.  Every other node is rebuilt only when a child changed."""
    memo: Dict[Node, Node] = {}
    stack = [(root, False)]
    while stack:
        n, ready = stack.pop()
        if n in memo:
            continue
        if not n.args:
            memo[n] = n
            continue
        if not ready:
            stack.append((n, True))
            stack.extend((c, False) for c in n.args if c not in memo)
            continue
        args = tuple(memo[c] for c in n.args)
        out = n if args == n.args else Node(n.op, n.width, args, n.param)
        if n.op == "ite" and n.width > 1:
            c, a, b = args
            if c.op in _MINMAX or c.op == "eq":
                x, y = c.args
                if (x, y) == (a, b) or (y, x) == (a, b):
                    same = (x, y) == (a, b)
                    if c.op == "eq":
                        out = b
                    else:
                        lo_hi = _MINMAX[c.op]
                        out = Node(lo_hi[0] if same else lo_hi[1], n.width, (x, y) if same else (x, y))
        memo[n] = out
    return memo[root]


class _Virt:
    """One device instruction before slot assignment."""
    __slots__ = ("op", "width", "args", "imm", "node")

    def __init__(self, op, width, args, imm=None, node=None):
        self.op, self.width, self.args, self.imm, self.node = op, width, args, imm, node


class PyCompiler:
    """The passes in Python: the reference implementation the native compiler
    (NativeCompiler, libmythgpu mg_cc_*) is tested against."""

    def __init__(self):
        self.var_index: Dict[str, int] = {}
        self.var_widths: List[int] = []
        self.const_index: Dict[int, int] = {}
        self.consts: List[int] = []
        self.max_slots = 0
        # arrays / functions / wide values -> 256-bit ops + table lookups (lower.py)
        self.lowering = Lowering()
        self.table_index: Dict[str, int] = {}

    # -- leaves ---------------------------------------------------------------
    def _leaf_ref(self, n: Node) -> int:
        if n.op == "const":
            i = self.const_index.get(n.param)
            if i is None:
                i = self.const_index[n.param] = len(self.consts)
                self.consts.append(n.param)
            return ref(REF_CONST, i)
        i = self.var_index.get(n.param)
        if i is None:
            i = self.var_index[n.param] = len(self.var_widths)
            self.var_widths.append(n.width)
        elif self.var_widths[i] != n.width:
            raise Unsupported(f"variable {n.param} used at two widths")
        return ref(REF_VAR, i)

    # -- scheduling -----------------------------------------------------------
    @staticmethod
    def _sizes(root: Node, size: Dict[Node, int]):
        order, st = [], [root]
        while st:
            x = st.pop()
            if x in size or x.op in ("const", "var"):
                continue
            size[x] = 0
            order.append(x)
            st.extend(x.args)
        for x in reversed(order):
            size[x] = 1 + sum(size.get(c, 0) for c in x.args)

    def _emit(self, n: Node, virts: List[_Virt], vid: Dict[Node, int], size: Dict[Node, int]):
        """Post-order emission of n's subtree; operands with bigger subtrees first so
        the last-computed operand is still in the accumulator."""
        stack = [(n, False)]
        while stack:
            x, ready = stack.pop()
            if x in vid or x.op in ("const", "var"):
                continue
            if x.width > 256 or any(c.width > 256 for c in x.args):
                raise Unsupported("bit-vector wider than 256 bits")
            if not ready:
                stack.append((x, True))
                kids = sorted((c for c in set(x.args) if c not in vid and c.op not in ("const", "var")),
                              key=lambda c: size.get(c, 0))
                for c in kids:            # pushed smallest-first => computed largest-first
                    stack.append((c, False))
                continue
            self._lower(x, virts, vid)

    def _schedule(self, root: Node) -> List[_Virt]:
        """The root conjunction And(c1..ck) is folded conjunct by conjunct (one
        running result in a slot) instead of computing every conjunct first."""
        size: Dict[Node, int] = {}
        self._sizes(root, size)
        virts: List[_Virt] = []
        vid: Dict[Node, int] = {}
        conj = list(root.args) if root.op == "and" else [root]
        running = None
        for c in conj:
            self._emit(c, virts, vid, size)
            cur = ("v", vid[c]) if c in vid else c
            if running is None:
                if not isinstance(cur, tuple):
                    virts.append(_Virt("copy", c.width, [c]))
                    cur = ("v", len(virts) - 1)
                running = cur
            else:
                virts.append(_Virt("and", 1, [running, cur]))
                running = ("v", len(virts) - 1)
        if root.op == "and" and conj:
            vid[root] = running[1]
        return virts

    def _lower(self, x: Node, virts: List[_Virt], vid: Dict[Node, int]):
        def arg(c):
            return ("v", vid[c]) if c in vid else c

        op = x.op
        if op in ("and", "or") and len(x.args) > 2:
            acc = arg(x.args[0])
            for c in x.args[1:]:
                virts.append(_Virt(op, 1, [acc, arg(c)]))
                acc = ("v", len(virts) - 1)
            vid[x] = len(virts) - 1
            return
        if op in ("and", "or") and len(x.args) == 1:
            virts.append(_Virt("copy", 1, [arg(x.args[0])]))
        elif op == "zero_extend" and x.args[0] in vid:
            # values are kept masked to their width, so zero-extending a computed
            # value changes no limb: the node aliases its operand's instruction
            vid[x] = vid[x.args[0]]
            return
        elif op == "extract":
            virts.append(_Virt("extract", x.width, [arg(x.args[0])], imm=x.param[1]))
        elif op == "sign_extend":
            virts.append(_Virt("sign_extend", x.width, [arg(x.args[0])], imm=x.args[0].width))
        elif op == "concat":
            virts.append(_Virt("concat", x.width, [arg(x.args[0]), arg(x.args[1])], imm=x.args[1].width))
        elif op in _CMP:
            virts.append(_Virt(op, 1, [arg(x.args[0]), arg(x.args[1])], imm=x.args[0].width))
        elif op == "tab":
            name, part, lo = x.param
            t = self.table_index.get(name)
            if t is None:
                t = self.table_index[name] = len(self.table_index)
            virts.append(_Virt("tab", x.width, [arg(x.args[0]), arg(x.args[1])],
                               imm=t | (part << TAB_PART_SHIFT) | (lo << TAB_LO_SHIFT)))
        elif op in OPCODE:
            virts.append(_Virt(op, x.width, [arg(c) for c in x.args]))
        else:
            raise Unsupported(f"operation {op} is not evaluated on the device")
        vid[x] = len(virts) - 1

    # -- slots + encoding -----------------------------------------------------
    def compile(self, root: Node) -> np.ndarray:
        root = _fold_select(self.lowering.lower(root))
        virts = self._schedule(root)
        n = len(virts)
        uses: Dict[int, List[Tuple[int, int]]] = {}
        for i, v in enumerate(virts):
            for k, a in enumerate(v.args):
                if isinstance(a, tuple):
                    uses.setdefault(a[1], []).append((i, k))
        # a result lives only in the accumulator when its single reader is the next
        # instruction, at a position the accumulator may take (_acc_ok)
        needs_slot = {j for j, us in uses.items()
                      if len(us) > 1 or any(i != j + 1 or not _acc_ok(virts[i].op, k) for i, k in us)}
        last_use = {j: max(i for i, _ in uses[j]) for j in needs_slot}
        slot_of: Dict[int, int] = {}
        free = list(range(MAX_SLOTS - 1, -1, -1))
        expiring: Dict[int, List[int]] = {}
        for i in range(n):
            for s in expiring.pop(i, []):
                free.append(s)
            if i in needs_slot:
                if not free:
                    raise Unsupported("constraint set needs more than 8 live values")
                s = free.pop()
                slot_of[i] = s
                self.max_slots = max(self.max_slots, s + 1)
                # the slot frees after its last reader has fetched its operands
                expiring.setdefault(last_use[i] + 1, []).append(s)
        out = np.zeros((n, 4), dtype=np.uint32)
        for i, v in enumerate(virts):
            refs = []
            op = v.op
            for k, a in enumerate(v.args):
                if isinstance(a, tuple):
                    j = a[1]
                    # the previous instruction's result, still in the accumulator
                    acc = j == i - 1 and (k == 0 or j not in slot_of)
                    refs.append(ref(REF_ACC, 0) if acc else ref(REF_SLOT, slot_of[j]))
                else:
                    refs.append(self._leaf_ref(a))
            if len(refs) > 1 and refs[1] >> 30 == REF_ACC:
                refs[0], refs[1] = refs[1], refs[0]          # the accumulator becomes operand A
                op = op if op in _COMMUTATIVE else _SWAPPED[op]
            assert all(r >> 30 != REF_ACC for r in refs[1:]), "accumulator past operand A"
            w = [enc_w0(op, v.width, slot_of.get(i)), 0, 0, 0]
            for k, r in enumerate(refs):
                w[1 + k] = r
            if v.op in ("extract", "sign_extend"):
                w[2] = v.imm
            elif v.op in ("concat", "rconcat") or v.op in _CMP or v.op == "tab":
                w[3] = v.imm
            out[i] = w
        if n > TILE_INSNS:
            raise Unsupported("program longer than one LDS tile")
        return out


class NativeCompiler(PyCompiler):
    """The same compiler with every pass after lowering in libmythgpu
    (csrc/cc.h through mg_cc_*): the lowered DAG's nodes are registered once
    each into the library's node table (a calldata word or a store chain
    shared by many conjuncts crosses once), leaves get their model-pool /
    constant-pool indices here, and each conjunct's program comes back from
    one call.  Lowering (arrays, uninterpreted functions, wide values ->
    256-bit ops and table lookups) stays in lower.py."""

    _VAR, _CONST, _BAD = 0x1000, 0x1001, 0xFFFF

    def __init__(self):
        super().__init__()
        import ctypes
        from .. import native
        self._ct = ctypes
        self._lib = native.load()
        self._cc = ctypes.c_void_p()
        if self._lib.mg_cc_open(ctypes.byref(self._cc)) != 0:
            raise native.MythGpuError("mg_cc_open failed")
        self._ids: Dict[Node, int] = {}
        self._buf = np.zeros((TILE_INSNS, 4), dtype=np.uint32)
        self._n = ctypes.c_uint32(0)
        self._ms = ctypes.c_uint32(0)

    def __del__(self):
        cc = getattr(self, "_cc", None)
        if cc:
            self._lib.mg_cc_close(cc)
            self._cc = None

    def _row(self, x: Node) -> Tuple[int, int]:
        """(op, imm) of a node for the library; _BAD for a node no program may
        contain (a variable used at two widths, an operation the device lacks)."""
        op = x.op
        if op == "const":
            i = self.const_index.get(x.param)
            if i is None:
                i = self.const_index[x.param] = len(self.consts)
                self.consts.append(x.param)
            return self._CONST, i
        if op == "var":
            i = self.var_index.get(x.param)
            if i is None:
                i = self.var_index[x.param] = len(self.var_widths)
                self.var_widths.append(x.width)
            elif self.var_widths[i] != x.width:
                return self._BAD, 0
            return self._VAR, i
        code = OPCODE.get(op)
        if code is None or op in ("bvumin", "bvumax", "bvsmin", "bvsmax", "bvrsub", "rconcat"):
            return self._BAD, 0
        if op == "extract":
            return code, x.param[1]
        if op == "tab":
            name, part, lo = x.param
            t = self.table_index.get(name)
            if t is None:
                t = self.table_index[name] = len(self.table_index)
            return code, t | (part << TAB_PART_SHIFT) | (lo << TAB_LO_SHIFT)
        return code, 0

    def _register(self, root: Node) -> int:
        ids = self._ids
        if root in ids:
            return ids[root]
        new: List[Node] = []
        local: Dict[Node, int] = {}
        stack = [(root, False)]
        while stack:
            x, ready = stack.pop()
            if x in ids or x in local:
                continue
            if not ready:
                stack.append((x, True))
                stack.extend((c, False) for c in x.args if c not in ids and c not in local)
                continue
            local[x] = len(new)
            new.append(x)
        flat: List[int] = []
        args: List[int] = []
        row = self._row
        for x in new:
            op, imm = row(x)
            flat += (op, x.width, len(args), len(x.args), imm)
            for c in x.args:
                j = local.get(c)
                args.append(ids[c] if j is None else (0x80000000 | j))
        rows = np.array(flat, dtype=np.uint32)
        a = np.array(args, dtype=np.uint32) if args else np.zeros(1, dtype=np.uint32)
        out = np.zeros(len(new), dtype=np.uint32)
        rc = self._lib.mg_cc_add(self._cc, rows.ctypes.data, len(new), a.ctypes.data, len(args), out.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"mg_cc_add: {self._lib.mg_cc_error(self._cc).decode()}")
        for x, i in zip(new, out.tolist()):
            ids[x] = i
        return ids[root]

    def compile(self, root: Node) -> np.ndarray:
        low = self.lowering.lower(root)
        rid = self._register(low)
        ct = self._ct
        self._ms.value = self.max_slots
        rc = self._lib.mg_cc_compile(self._cc, rid, self._buf.ctypes.data, TILE_INSNS, ct.byref(self._n),
                                     ct.byref(self._ms))
        if rc == -6:
            raise Unsupported(self._lib.mg_cc_error(self._cc).decode())
        if rc != 0:
            raise RuntimeError(f"mg_cc_compile: {self._lib.mg_cc_error(self._cc).decode()}")
        self.max_slots = int(self._ms.value)
        return self._buf[: self._n.value].copy()


# the product compiler: native passes (libmythgpu); PyCompiler is their reference
Compiler = NativeCompiler


def compile_sets(sets: Sequence[Sequence], compiler: PyCompiler = None) -> Tuple[ProgramBatch, List[int]]:
    """Compile constraint sets (each a list of Bool / Node) into one ProgramBatch.
    Returns the batch and the indices of the sets it contains (unsupported sets
    are left out and must go to z3)."""
    c = compiler or Compiler()
    progs, kept = [], []
    for k, s in enumerate(sets):
        raws = [x.raw if isinstance(x, Bool) else x for x in s]
        raws = [r for r in raws if r is not TRUE]
        root = raws[0] if len(raws) == 1 else (Node("and", 1, tuple(raws)) if raws else TRUE)
        try:
            progs.append(c.compile(root))
            kept.append(k)
        except Unsupported:
            continue
    off = np.zeros(len(progs) + 1, dtype=np.uint32)
    if progs:
        off[1:] = np.cumsum([p.shape[0] for p in progs])
        insns = np.concatenate(progs)
    else:
        insns = np.zeros((0, 4), dtype=np.uint32)
    consts = np.stack([limbs(x) for x in c.consts]) if c.consts else np.zeros((0, 8), np.uint32)
    names = [None] * len(c.var_widths)
    for name, i in c.var_index.items():
        names[i] = name
    tables = [None] * len(c.table_index)
    for name, t in c.table_index.items():
        tables[t] = c.lowering.tables[name]
    return ProgramBatch(insns, off, consts, max(c.max_slots, 1), names, list(c.var_widths),
                        tables), kept


def batch_from(c: "PyCompiler", progs: List[np.ndarray]) -> ProgramBatch:
    """A ProgramBatch of programs compiled by one (persistent) Compiler: its
    variable, constant and table index spaces only grow, so programs compiled
    for earlier batches stay valid in later ones."""
    off = np.zeros(len(progs) + 1, dtype=np.uint32)
    if progs:
        off[1:] = np.cumsum([p.shape[0] for p in progs])
        insns = np.concatenate(progs)
    else:
        insns = np.zeros((0, 4), dtype=np.uint32)
    # the compiler's constant limbs and variable names, extended by what it added
    # since the last batch (its index spaces only grow)
    cache = getattr(c, "_batch_cache", None)
    if cache is None:
        cache = c._batch_cache = {"consts": np.zeros((0, 8), np.uint32), "names": []}
    if cache["consts"].shape[0] < len(c.consts):
        new = np.stack([limbs(x) for x in c.consts[cache["consts"].shape[0]:]])
        cache["consts"] = np.concatenate([cache["consts"], new])
    consts = cache["consts"]
    names = cache["names"]
    if len(names) < len(c.var_widths):
        names.extend([None] * (len(c.var_widths) - len(names)))
        for name, i in c.var_index.items():
            names[i] = name
    tables = [None] * len(c.table_index)
    for name, t in c.table_index.items():
        tables[t] = c.lowering.tables[name]
    return ProgramBatch(insns, off, consts, max(c.max_slots, 1), list(names), list(c.var_widths), tables)
