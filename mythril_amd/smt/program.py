"""Device formats of kernel 2: compiled constraint programs and candidate models.

A ``ProgramBatch`` is the host image of mg_dag_batch (include/mythgpu.h); a
``ModelPool`` the host image of mg_model_batch.  Instruction encoding matches
bv_eval.cuh (4 x u32: op | width<<8 | store<<17 | slot<<18, then three operand
refs kind<<30 | index, or immediates).
"""
from __future__ import annotations

import ctypes
import itertools
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

OPS = ["copy", "bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod",
       "bvand", "bvor", "bvxor", "bvnot", "bvneg", "bvshl", "bvlshr", "bvashr",
       "eq", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
       "and", "or", "xor", "not", "implies", "ite", "extract", "concat", "zero_extend",
       "sign_extend", "bvadd_noovfl_u", "bvumul_noovfl", "bvsub_noudfl_u", "distinct", "tab",
       # compiler-internal: ite(cmp(x, y), x, y) folded by flatten._fold_select
       "bvumin", "bvumax", "bvsmin", "bvsmax",
       # compiler-internal operand-swapped forms (the accumulator is only ever
       # operand A, bv_eval.cuh): bvrsub(a, b) = b - a; rconcat(a, b) = concat(b, a)
       # with the immediate the width of a
       "bvrsub", "rconcat"]
OPCODE = {name: i for i, name in enumerate(OPS)}
UNARY = {"copy", "bvnot", "bvneg", "not", "extract", "zero_extend", "sign_extend"}
REF_ACC, REF_SLOT, REF_VAR, REF_CONST = 0, 1, 2, 3
TAB_PART_SHIFT, TAB_LO_SHIFT, TAB_INDEX_MASK = 20, 21, (1 << 20) - 1
MAX_SLOTS = 16       # kernel 2's 4-bit slot field (BV_MAX_SLOTS)
TILE_INSNS = 2048


# operand references per op (bv_upload: ite 3, one-operand ops 1, the rest 2)
_NREF = np.array([3 if op == "ite" else 1 if op in UNARY else 2 for op in OPS], dtype=np.int64)
def _reads(ins: np.ndarray):
    """(opcodes, per-operand variable masks, variables read, table-read mask,
    tables read) of an instruction array."""
    op = (ins[:, 0] & 0xFF).astype(np.int64)
    nref = _NREF[np.minimum(op, len(_NREF) - 1)]
    isvar = [(nref > k) & ((ins[:, 1 + k] >> 30) == REF_VAR) for k in range(3)]
    used = np.unique(np.concatenate([ins[m, 1 + k] & 0x3FFFFFFF for k, m in enumerate(isvar)]))
    istab = op == OPCODE["tab"]
    tabs = np.unique(ins[istab, 3] & TAB_INDEX_MASK) if istab.any() else np.zeros(0, dtype=np.uint32)
    return op, isvar, used, istab, tabs


def read_sets(batch: "ProgramBatch"):
    """(variable indices, table indices) the batch's programs read."""
    ins = np.asarray(batch.insns, dtype=np.uint32)
    if ins.shape[0] == 0:
        return frozenset(), frozenset()
    _, _, used, _, tabs = _reads(ins)
    return frozenset(used.tolist()), frozenset(tabs.tolist())


def compact_vars(batch: "ProgramBatch") -> "ProgramBatch":
    """The batch with its variables and tables renumbered to those its programs
    read (a persistent compiler's batches carry every variable and table it has
    seen; a pool built from model dicts then serialises all of them).  Same
    programs, same values: only the index spaces shrink."""
    ins = np.asarray(batch.insns, dtype=np.uint32)
    if ins.shape[0] == 0:
        return batch
    op, isvar, used, istab, tabs = _reads(ins)
    if used.size == len(batch.var_names) and tabs.size == len(batch.tables):
        return batch
    out = ins.copy()
    vmap = np.zeros(max(len(batch.var_names), 1), dtype=np.uint32)
    vmap[used] = np.arange(used.size, dtype=np.uint32)
    for k, m in enumerate(isvar):
        out[m, 1 + k] = (np.uint32(REF_VAR) << np.uint32(30)) | vmap[ins[m, 1 + k] & 0x3FFFFFFF]
    if tabs.size:
        tmap = np.zeros(max(len(batch.tables), 1), dtype=np.uint32)
        tmap[tabs] = np.arange(tabs.size, dtype=np.uint32)
        imm = ins[istab, 3]
        out[istab, 3] = (imm & ~np.uint32(TAB_INDEX_MASK)) | tmap[imm & TAB_INDEX_MASK]
    return ProgramBatch(out, batch.prog_off, batch.consts, batch.n_slots,
                        [batch.var_names[i] for i in used.tolist()],
                        [batch.var_widths[i] for i in used.tolist()],
                        [batch.tables[i] for i in tabs.tolist()])


def ref(kind: int, idx: int) -> int:
    return (kind << 30) | idx


def enc_w0(op: str, width: int, store_slot: Optional[int] = None) -> int:
    w = OPCODE[op] | (width << 8)
    if store_slot is not None:
        w |= (1 << 17) | (store_slot << 18)
    return w


@dataclass
class ProgramBatch:
    insns: np.ndarray          # (total, 4) uint32
    prog_off: np.ndarray       # (n_dags + 1,) uint32
    consts: np.ndarray         # (n_consts, 8) uint32 little-endian limbs
    n_slots: int
    var_names: List[str] = field(default_factory=list)
    var_widths: List[int] = field(default_factory=list)
    tables: List = field(default_factory=list)      # lower.TableSig per table index

    @property
    def n_dags(self) -> int:
        return int(self.prog_off.shape[0] - 1)

    def program(self, d: int) -> np.ndarray:
        return self.insns[self.prog_off[d]:self.prog_off[d + 1]]

    def c_struct(self):
        from ..native import MgDagBatch
        self.insns = np.ascontiguousarray(self.insns, dtype=np.uint32)
        self.prog_off = np.ascontiguousarray(self.prog_off, dtype=np.uint32)
        self.consts = np.ascontiguousarray(self.consts, dtype=np.uint32)
        if self.consts.shape[0] == 0:
            self.consts = np.zeros((1, 8), dtype=np.uint32)
        s = MgDagBatch(self.n_dags, max(self.n_slots, 1), self.prog_off.ctypes.data,
                       self.insns.ctypes.data, self.consts.ctypes.data,
                       int(self.consts.shape[0]))
        return s


class ArrayInterp:
    """A model's interpretation of a symbolic array: default + entries
    (z3's K(default) + stores / as-array)."""
    __slots__ = ("default", "_entries", "dense")

    def __init__(self, default: int = 0, entries: Optional[Dict[int, int]] = None,
                 dense: Optional[bytes] = None):
        self.default = default
        # dense: entries 0..len-1 as bytes (a witness seed's calldata), turned
        # into the entry dict only when something reads `entries`
        self.dense = dense if entries is None else None
        self._entries = dict(entries) if entries is not None else (None if dense is not None else {})

    @property
    def entries(self) -> Dict[int, int]:
        if self._entries is None:
            self._entries = dict(enumerate(self.dense))
        return self._entries

    def untouched_dense(self) -> Optional[bytes]:
        """The dense bytes while no one has taken the entry dict (which may then
        have been changed), else None."""
        return self.dense if self._entries is None else None


class FuncInterp:
    """A model's interpretation of an uninterpreted function: entries (argument
    tuple -> value) + else value."""
    __slots__ = ("else_value", "entries")

    def __init__(self, else_value: int = 0, entries: Optional[Dict[tuple, int]] = None):
        self.else_value = else_value
        self.entries = dict(entries or {})


def model_value(model: Dict[str, object], name: str) -> int:
    """A variable's value in a model dict; a constant-index select variable
    (lower.select_var: ``array<SEP>index``) reads the array interpretation's
    entry or default.  Anything absent is 0 (z3 model_completion)."""
    x = model.get(name)
    if x is None and "\x1f" in name:
        arr, _, k = name.partition("\x1f")
        interp = model.get(arr)
        if isinstance(interp, ArrayInterp):
            return interp.entries.get(int(k), interp.default)
        return 0
    return x if isinstance(x, int) else 0


def _wide_limbs(x: int) -> np.ndarray:
    """512-bit value -> 16 little-endian u32 limbs."""
    return np.frombuffer((x & ((1 << 512) - 1)).to_bytes(64, "little"), dtype="<u4")


@dataclass
class ModelPool:
    """values[v, m] = value of variable v in model m (256-bit limbs), models in
    most-recently-used-first order (support_utils.py:62-63).  Tables hold the
    models' array / function interpretations: for table t and model m the
    entries tab_entries[tab_start[t, m] : + tab_count[t, m]] (each key k0, k1 and
    a 512-bit value, 32 u32) and the default / else value tab_default[t, m]."""
    values: np.ndarray         # (n_vars, n_models, 8) uint32
    tab_start: Optional[np.ndarray] = None     # (n_tables, n_models) uint32
    tab_count: Optional[np.ndarray] = None     # (n_tables, n_models) uint32
    tab_entries: Optional[np.ndarray] = None   # (n_entries, 32) uint32
    tab_default: Optional[np.ndarray] = None   # (n_tables, n_models, 16) uint32

    @property
    def n_models(self) -> int:
        return int(self.values.shape[1])

    @property
    def n_vars(self) -> int:
        return int(self.values.shape[0])

    @property
    def n_tables(self) -> int:
        return 0 if self.tab_start is None else int(self.tab_start.shape[0])

    def c_struct(self):
        from ..native import MgModelBatch
        self.values = np.ascontiguousarray(self.values, dtype=np.uint32)
        if self.n_tables == 0:
            return MgModelBatch(self.n_models, self.n_vars, self.values.ctypes.data, 0, None, None,
                                None, 0, None)
        for f in ("tab_start", "tab_count", "tab_entries", "tab_default"):
            setattr(self, f, np.ascontiguousarray(getattr(self, f), dtype=np.uint32))
        if self.tab_entries.shape[0] == 0:
            self.tab_entries = np.zeros((1, 32), dtype=np.uint32)
        return MgModelBatch(self.n_models, self.n_vars, self.values.ctypes.data, self.n_tables,
                            self.tab_start.ctypes.data, self.tab_count.ctypes.data,
                            self.tab_entries.ctypes.data, int(self.tab_entries.shape[0]),
                            self.tab_default.ctypes.data)

    @staticmethod
    def from_dicts(models: List[Dict[str, object]], var_names: List[str], var_widths: List[int],
                   tables: Optional[List] = None, reads=None):
        """models: name -> int for variables, ArrayInterp / FuncInterp for tables;
        anything absent is completed with 0 (z3 model_completion).  reads: the
        (variable, table) index sets the programs evaluated on the pool read
        (read_sets); the others are left zero / empty, as no program sees them."""
        vals = np.zeros((max(len(var_names), 1), max(len(models), 1), 8), dtype=np.uint32)
        rv, rt = reads if reads is not None else (None, None)
        for v, (name, w) in enumerate(zip(var_names, var_widths)):
            if rv is not None and v not in rv:
                continue
            # one bytes join per variable: the per-element numpy writes cost
            # more than the values themselves
            mask = (1 << w) - 1
            raw = b"".join((model_value(model, name) & mask).to_bytes(32, "little") for model in models)
            if raw:
                vals[v, :len(models)] = np.frombuffer(raw, dtype="<u4").reshape(len(models), 8)
        pool = ModelPool(vals)
        tables = tables or []
        if tables:
            nm = max(len(models), 1)
            start = np.zeros((len(tables), nm), dtype=np.uint32)
            count = np.zeros((len(tables), nm), dtype=np.uint32)
            default = np.zeros((len(tables), nm, 16), dtype=np.uint32)
            rows: List[bytes] = []
            M256 = (1 << 256) - 1
            M512 = (1 << 512) - 1
            for t, sig in enumerate(tables):
                for m, model in enumerate(models):
                    interp = model.get(sig.name) if rt is None or t in rt else None
                    start[t, m] = len(rows)
                    if isinstance(interp, ArrayInterp):
                        default[t, m] = _wide_limbs(interp.default)
                        items = [((k,), v) for k, v in interp.entries.items()]
                    elif isinstance(interp, FuncInterp):
                        default[t, m] = _wide_limbs(interp.else_value)
                        items = list(interp.entries.items())
                    else:
                        items = []
                    for args, v in items:
                        k0, k1 = sig.key_chunks(tuple(args))
                        rows.append((k0 & M256).to_bytes(32, "little") + (k1 & M256).to_bytes(32, "little") +
                                    (v & M512).to_bytes(64, "little"))
                    count[t, m] = len(rows) - start[t, m]
            entries = (np.frombuffer(b"".join(rows), dtype="<u4").reshape(len(rows), 32).copy() if rows
                       else np.zeros((0, 32), dtype=np.uint32))
            pool.tab_start, pool.tab_count, pool.tab_entries, pool.tab_default = \
                start, count, entries, default
        return pool


def limbs(x: int) -> np.ndarray:
    return np.frombuffer((x & ((1 << 256) - 1)).to_bytes(32, "little"), dtype="<u4").copy()


def concat_pools(a: ModelPool, b: ModelPool) -> ModelPool:
    """Pool a's models followed by pool b's (same variables and tables)."""
    out = ModelPool(np.concatenate([a.values, b.values], axis=1))
    if a.n_tables:
        shift = np.uint32(a.tab_entries.shape[0])
        out.tab_start = np.concatenate([a.tab_start, b.tab_start + shift], axis=1)
        out.tab_count = np.concatenate([a.tab_count, b.tab_count], axis=1)
        out.tab_entries = np.concatenate([a.tab_entries, b.tab_entries], axis=0)
        out.tab_default = np.concatenate([a.tab_default, b.tab_default], axis=1)
    return out


class PoolColumns:
    """A fixed list of model assignments, laid out once per variable and per
    table: ``pool(var_names, var_widths, tables)`` assembles a ModelPool from
    cached columns (the witness seeds are rebuilt only when they change)."""

    def __init__(self, assigns: List[Dict[str, object]], revision=None):
        self.assigns = assigns
        self._vars: Dict[tuple, np.ndarray] = {}
        self._tabs: Dict[tuple, tuple] = {}
        self._dense_cache: Dict[str, tuple] = {}
        self._mat: Optional[np.ndarray] = None   # rows of the last pool's variables
        self._mat_keys: List[tuple] = []
        self._mat_revs: List[object] = []
        # revision(name) -> a value that changes whenever any assignment's
        # interpretation of `name` changes (None: interpretations never change)
        self.revision = revision or (lambda name: 0)

    def _var(self, name: str, w: int) -> np.ndarray:
        sel = "\x1f" in name
        rev = self.revision(name.partition("\x1f")[0]) if sel else 0
        got = self._vars.get((name, w))
        if got is None or got[0] != rev:
            mask = (1 << w) - 1
            k = int(name.partition("\x1f")[2]) if sel else -1
            dense = self._dense(name.partition("\x1f")[0], rev) if sel and w <= 64 and k < self.DENSE_KEYS else None
            if dense is not None:
                mat, dflt = dense
                v = (mat[:, k] if k < mat.shape[1] else dflt) & np.uint64(mask)
                col = np.zeros((len(self.assigns), 8), dtype=np.uint32)
                col[:, 0] = (v & np.uint64(0xFFFFFFFF)).astype(np.uint32)
                col[:, 1] = (v >> np.uint64(32)).astype(np.uint32)
                got = self._vars[(name, w)] = (rev, col)
                return col
            if sel:
                raw = b"".join((model_value(a, name) & mask).to_bytes(32, "little") for a in self.assigns)
            else:
                raw = b"".join(((x if isinstance(x := a.get(name, 0), int) else 0) & mask).to_bytes(32, "little")
                               for a in self.assigns)
            got = self._vars[(name, w)] = (rev, np.frombuffer(raw, dtype="<u4").reshape(-1, 8).astype(np.uint32))
        return got[1]

    DENSE_KEYS = 4096

    def _dense(self, arr: str, rev):
        """Every model's interpretation of array ``arr`` at small indices as one
        (n_models, K) uint64 matrix plus the defaults (the witness seeds'
        calldata bytes): a constant-index select column is then one numpy
        slice instead of a dictionary lookup per model.  None when a value
        does not fit 64 bits."""
        got = self._dense_cache.get(arr)
        if got is not None and got[0] == rev:
            return got[1]
        nm = len(self.assigns)
        interps = [a.get(arr) for a in self.assigns]
        raws = [it.untouched_dense() if isinstance(it, ArrayInterp) else None for it in interps]
        if nm and all(r is not None for r in raws) and all(it.default < 256 for it in interps):
            # every model holds the array as bytes (the seeds' calldata): one scatter
            lens = np.fromiter(map(len, raws), dtype=np.int64, count=nm)
            dflt = np.fromiter((it.default for it in interps), dtype=np.uint64, count=nm)
            top = int(lens.max()) if nm else 0
            mat = np.repeat(dflt[:, None], top, axis=1)
            if top:
                flat = np.frombuffer(b"".join(raws), dtype=np.uint8)
                rows = np.repeat(np.arange(nm), lens)
                starts = np.concatenate(([0], np.cumsum(lens)[:-1]))
                cols = np.arange(flat.size) - np.repeat(starts, lens)
                mat[rows, cols] = flat
            out = (mat[:, :self.DENSE_KEYS], dflt)
            self._dense_cache[arr] = (rev, out)
            return out
        keys, vals, dflt = [], [], np.zeros(nm, dtype=np.uint64)
        top = 0
        for m, a in enumerate(self.assigns):
            interp = a.get(arr)
            if not isinstance(interp, ArrayInterp):
                keys.append(()), vals.append(())
                continue
            if interp.default >> 64:
                self._dense_cache[arr] = (rev, None)
                return None
            dflt[m] = interp.default
            raw = interp.untouched_dense()
            if raw is not None:
                ks = slice(0, min(len(raw), self.DENSE_KEYS))
                keys.append(ks), vals.append(np.frombuffer(raw, dtype=np.uint8)[ks])
                top = max(top, ks.stop)
                continue
            ks = [k for k in interp.entries if k < self.DENSE_KEYS]
            vs = [interp.entries[k] for k in ks]
            if vs and max(vs) >> 64:
                self._dense_cache[arr] = (rev, None)
                return None
            keys.append(ks), vals.append(vs)
            if ks:
                top = max(top, max(ks) + 1)
        mat = np.repeat(dflt[:, None], top, axis=1)
        for m in range(nm):
            if isinstance(keys[m], slice) or keys[m]:
                mat[m, keys[m]] = vals[m]
        out = (mat, dflt)
        self._dense_cache[arr] = (rev, out)
        return out

    def _tab(self, sig) -> tuple:
        """(start, count, entries, default) of one table over every model.
        Interpretations only grow (witness seeds gain entries, never change
        one), so a revision serialises only each model's new entries."""
        key = (sig.name, sig.kind, sig.domain, sig.range)
        rev = self.revision(sig.name)
        got = self._tabs.get(key)
        if got is not None and got[0] == rev:
            return got[1]
        nm = len(self.assigns)
        if got is None:
            ser = [bytearray() for _ in range(nm)]      # per model: serialised rows
            done = [0] * nm                              # entries serialised
            dflt = [None] * nm
        else:
            ser, done, dflt = got[2]
        M256_, M512_ = (1 << 256) - 1, (1 << 512) - 1
        for m, a in enumerate(self.assigns):
            interp = a.get(sig.name)
            raw = interp.untouched_dense() if isinstance(interp, ArrayInterp) else None
            if raw is not None:
                # rows (key, 0, byte) of a dense interpretation, in key order (the
                # entry dict's insertion order when it is taken later)
                rows = np.zeros((len(raw), 32), dtype="<u4")
                rows[:, 0] = np.arange(len(raw), dtype=np.uint32)
                rows[:, 16] = np.frombuffer(raw, dtype=np.uint8)
                ser[m], done[m], dflt[m] = bytearray(rows.tobytes()), len(raw), interp.default
                continue
            if isinstance(interp, ArrayInterp):
                d, ent, arr = interp.default, interp.entries, True
            elif isinstance(interp, FuncInterp):
                d, ent, arr = interp.else_value, interp.entries, False
            else:
                d, ent, arr = 0, {}, False
            if len(ent) < done[m] or dflt[m] != d:       # not append-only: start over
                ser[m], done[m] = bytearray(), 0
            dflt[m] = d
            if len(ent) > done[m]:
                # a row is (k0, k1, value): for a one-argument key of up to 512 bits
                # k0 | k1 << 256 is the key itself (TableSig.key_chunks), so the
                # first 64 bytes are the key's little-endian bytes
                new = itertools.islice(ent.items(), done[m], None)
                if arr:
                    ser[m] += b"".join((k & M512_).to_bytes(64, "little") + (v & M512_).to_bytes(64, "little")
                                       for k, v in new)
                else:
                    ser[m] += b"".join(
                        ((k[0] & M512_).to_bytes(64, "little") if len(k) == 1 else
                         (k[0] & M256_).to_bytes(32, "little") + (k[1] & M256_).to_bytes(32, "little")) +
                        (v & M512_).to_bytes(64, "little") for k, v in new)
                done[m] = len(ent)
        count = np.array(done, dtype=np.uint32)
        start = np.zeros(nm, dtype=np.uint32)
        if nm > 1:
            start[1:] = np.cumsum(count[:-1])
        entries = np.frombuffer(b"".join(ser), dtype="<u4").reshape(-1, 32).astype(np.uint32)
        default = np.frombuffer(b"".join(((x or 0) & M512_).to_bytes(64, "little") for x in dflt),
                                dtype="<u4").reshape(nm, 16).astype(np.uint32)
        out = (start, count, entries, default)
        self._tabs[key] = (rev, out, (ser, done, dflt))
        return out

    def pool(self, var_names: List[str], var_widths: List[int], tables: Optional[List] = None) -> ModelPool:
        nm = len(self.assigns)
        nv = len(var_names)
        # one persistent (variables x models) matrix: a persistent compiler's
        # variable list only grows, so a launch fills the rows of new variables
        # and of select variables whose array changed, not every row again
        if self._mat is None or self._mat.shape[0] < max(nv, 1):
            grown = np.zeros((max(nv, 1, 2 * (0 if self._mat is None else self._mat.shape[0])), max(nm, 1), 8),
                             dtype=np.uint32)
            if self._mat is not None:
                grown[:self._mat.shape[0]] = self._mat
            self._mat = grown
        keys, revs = self._mat_keys, self._mat_revs
        for v, (name, w) in enumerate(zip(var_names, var_widths)):
            arr = name.partition("\x1f")[0] if "\x1f" in name else None
            rev = self.revision(arr) if arr is not None else 0
            if v < len(keys) and keys[v] == (name, w) and revs[v] == rev:
                continue
            self._mat[v, :nm] = self._var(name, w)
            if v < len(keys):
                keys[v], revs[v] = (name, w), rev
            else:
                keys.append((name, w))
                revs.append(rev)
        out = ModelPool(self._mat[:max(nv, 1)])
        if tables:
            parts = [self._tab(sig) for sig in tables]
            starts, counts, defaults, ents, off = [], [], [], [], 0
            for st, ct, en, df in parts:
                starts.append(st + np.uint32(off))
                counts.append(ct)
                defaults.append(df)
                ents.append(en)
                off += en.shape[0]
            out.tab_start = np.stack(starts)
            out.tab_count = np.stack(counts)
            out.tab_default = np.stack(defaults)
            out.tab_entries = np.concatenate(ents, axis=0) if off else np.zeros((0, 32), dtype=np.uint32)
        return out
