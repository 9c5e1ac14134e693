"""Witness seeds: concrete transaction inputs as candidate models for kernel 2.

The reference's quick-sat (support_utils.py:34-68) can only answer with one of
the <= 100 models its SMT backend returned earlier.  Kernel 2 evaluates
thousands of candidates per constraint set for the price of a few, so a pool of
*concrete transaction inputs* -- the calldata, sender, call value and initial
storage a concrete run of the contract would use -- proves "SAT" for every path
such an input drives, before any solver is asked (the prefilter
may only answer SAT with a model; a miss falls through unchanged).  The pool is
consulted only where get_model would call the backend (solver.ModelCache
.check_seeds), and a seed it returns is checked against the whole query, the
keccak conjunct included, on the device.

A seed assigns, for every symbolic transaction id N the queries mention,
``N_calldata`` (a byte array: a dispatcher selector of the code, then argument
words drawn from zero / small / actor address / random address / random word /
all-ones), ``N_calldatasize``, ``sender_N`` (one of the ACTORS,
transaction/symbolic.py:28-40), ``call_valueN`` (mostly 0) and ``gas_priceN``;
the symbolic storage arrays start at 0.  Keccak functions are completed per
seed so the KeccakFunctionManager axioms hold (keccak_function_manager.py:
116-179): each registered symbolic input x evaluates under the seed to v, and
keccak256_N(v) is keccak(c) when v is a registered concrete input c, else a
fresh multiple of 64 inside N's interval, with the inverse mapping back; and
Power is the true power at every concrete EXP registered (the constraints
exponent_function_manager.py:32-60 adds, with its 256**i table).
"""
from __future__ import annotations

import re
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from ..smt.expr import Node
from ..smt.keccak_manager import PART, KeccakFunctionManager, keccak_function_manager
from ..smt.program import ArrayInterp, FuncInterp
from ..smt.solver import Model, ModelRef
from .transaction import ACTORS

M256 = (1 << 256) - 1
_TX_VAR = re.compile(r"^(?:sender_(\d+)|call_value(\d+)|gas_price(\d+)|(\d+)_calldata(?:size)?)$")


def dispatch_selectors(code: bytes) -> List[int]:
    """The 4-byte constants a Solidity dispatcher compares the selector with
    (PUSH4 x; EQ)."""
    out, k = [], 0
    while k < len(code):
        op = code[k]
        if op == 0x63 and k + 6 <= len(code) and code[k + 5] == 0x14:
            out.append(int.from_bytes(code[k + 1:k + 5], "big"))
        k += 1 + (op - 0x5F if 0x60 <= op <= 0x7F else 0)
    return sorted(set(out))


class WitnessSeeds:
    """A fixed pool of `n` seed models over the transactions the queries name.

    ``models()`` returns the pool as solver Models, extended with the
    variables of newly seen transaction ids and completed for the keccak
    inputs registered so far (incrementally: values already computed are
    kept)."""

    def __init__(self, codes: Sequence[bytes], n: int = 1024, seed: int = 0x5EED5EED,
                 storage_names: Iterable[str] = (), manager: KeccakFunctionManager = keccak_function_manager,
                 balance_names: Iterable[str] = ()):
        self.n = n
        self.rng = np.random.default_rng(seed)
        sel = []
        for c in codes:
            sel.extend(dispatch_selectors(bytes(c)))
        self.selectors = sorted(set(sel)) or [0]
        self.storage_names = list(storage_names)
        self.km = manager
        self.assign: List[Dict[str, object]] = [{} for _ in range(n)]
        # balances (world_state.py:31-33 Array("balance")): every account starts
        # with the same balance, a few ether, mostly (reachable under
        # analysis/solver.py's 100 / 1000 ether bounds; 0 for some seeds)
        self.balance_names = list(balance_names)
        for m, a in enumerate(self.assign):
            for name in self.storage_names:
                a[name] = ArrayInterp(0, {})
            for name in self.balance_names:
                a[name] = ArrayInterp(0 if m % 8 == 7 else 10 ** (18 + m % 3), {})
        self.tx_ids: List[str] = []
        self._done: List[Dict[Node, int]] = [{} for _ in range(n)]   # keccak input -> value, per seed
        self._next: List[Dict[int, int]] = [{} for _ in range(n)]    # next free slot per input size
        self._models: Optional[List[Model]] = None
        self._epoch = None
        self._rev: Dict[str, int] = {}           # interpretation changes per name (PoolColumns)
        self._tx_top = -1
        self._sym_pts = 0                        # symbolic EXP points completed so far
        self._pw_seen: set = set()               # concrete EXP points entered into every seed
        self._cc_seen: set = set()               # concrete hashes entered into every seed

    def revision(self, name: str) -> int:
        return self._rev.get(name, 0)

    def _touch(self, name: str) -> None:
        self._rev[name] = self._rev.get(name, 0) + 1

    # -- transactions ------------------------------------------------------------------
    def add_tx(self, txid: str) -> None:
        if txid in self.tx_ids:
            return
        self.tx_ids.append(txid)
        self._touch(f"{txid}_calldata")
        actors = list(ACTORS.values())
        r = self.rng
        n = self.n
        # every seed's draws at once (numpy), then one pass to build the arrays
        nargs = r.integers(0, 4, n)
        use_sel = r.random(n) < 0.9
        sel = r.integers(0, len(self.selectors), n)
        junk = r.integers(0, 256, (n, 4), dtype=np.uint8)
        argb = self._args(actors, n * 3)
        cut = r.random(n) < 0.05
        cut_at = r.random(n)
        value_nz = r.random(n) >= 0.85
        values = r.integers(1, 1 << 20, n)
        gas = r.integers(0, 1 << 40, n)
        sel_bytes = [x.to_bytes(4, "big") for x in self.selectors]
        na = len(actors)
        for m, a in enumerate(self.assign):
            data = sel_bytes[int(sel[m])] if use_sel[m] else junk[m].tobytes()
            k = int(nargs[m])
            if k:
                data += argb[m * 3:m * 3 + k].tobytes()
            if cut[m] and data:
                data = data[:int(cut_at[m] * len(data))]
            a[f"{txid}_calldata"] = ArrayInterp(0, dense=data)
            a[f"{txid}_calldatasize"] = len(data)
            a[f"sender_{txid}"] = actors[m % na]
            a[f"call_value{txid}"] = int(values[m]) if value_nz[m] else 0
            a[f"gas_price{txid}"] = int(gas[m])

    def _args(self, actors, k: int) -> np.ndarray:
        """k argument words as (k, 32) big-endian bytes: zero, small, an actor, a
        random address, a random word or all ones."""
        r = self.rng
        u = r.random(k)
        small = r.integers(0, 1 << 16, k)
        who = r.integers(0, len(actors), k)
        raw = r.integers(0, 256, (k, 32), dtype=np.uint8)
        out = np.zeros((k, 32), dtype=np.uint8)
        sm = (u >= 0.15) & (u < 0.40)
        out[sm, 30] = (small[sm] >> 8).astype(np.uint8)
        out[sm, 31] = (small[sm] & 0xFF).astype(np.uint8)
        ac = (u >= 0.40) & (u < 0.60)
        table = np.frombuffer(b"".join(x.to_bytes(32, "big") for x in actors), dtype=np.uint8).reshape(-1, 32)
        out[ac] = table[who[ac]]
        ad = (u >= 0.60) & (u < 0.75)
        out[ad, 12:] = raw[ad, :20]
        wd = (u >= 0.75) & (u < 0.90)
        out[wd] = raw[wd]
        out[u >= 0.90] = 0xFF
        return out

    def note_query_vars(self, names: Iterable[str]) -> None:
        for name in names:
            mt = _TX_VAR.match(name)
            if mt:
                self.add_tx(next(g for g in mt.groups() if g is not None))

    # -- keccak completion --------------------------------------------------------------
    def _complete(self) -> None:
        km = self.km
        inputs = [x for xs in km.symbolic_inputs.values() for x in xs]
        concrete = {}
        for c, h in km.concrete_hashes.items():
            concrete[(c.size(), c.value)] = h.value
        if inputs:
            km.create_conditions()          # assigns the intervals in the reference's order
        from ..smt.exponent_manager import exponent_function_manager
        power = exponent_function_manager.concrete_points
        # an interpretation's revision changes only when entries are added to it
        # (PoolColumns re-serialises a table per revision)
        changed = set()
        # concrete points and hashes only accumulate: each is entered into the
        # seeds once (an entry a seed already holds is left as it is)
        new_pw = [(k, v) for k, v in power.items() if k not in self._pw_seen]
        new_cc = [(k, h) for k, h in concrete.items() if k not in self._cc_seen]
        for a in self.assign:
            pw = a.setdefault("Power", FuncInterp(0, {}))
            for be, v in new_pw:
                if be not in pw.entries:
                    pw.entries[be] = v
                    changed.add("Power")
            for (n, cv), h in new_cc:
                f = a.setdefault(f"keccak256_{n}", FuncInterp(0, {}))
                if (cv,) not in f.entries:
                    f.entries[(cv,)] = h
                    changed.add(f"keccak256_{n}")
                inv = a.setdefault(f"keccak256_{n}-1", FuncInterp(0, {}))
                if (h,) not in inv.entries:
                    inv.entries[(h,)] = cv
                    changed.add(f"keccak256_{n}-1")
        self._pw_seen.update(k for k, _ in new_pw)
        self._cc_seen.update(k for k, _ in new_cc)
        # inputs in registration order (an input may hash an earlier one's hash):
        # each evaluated under every seed at once, then entered into the seeds'
        # keccak tables
        for x in inputs:
            n = x.size()
            todo = [m for m in range(self.n) if x.raw not in self._done[m]]
            if not todo:
                continue
            vals = eval_all(x.raw, [self.assign[m] for m in todo])
            for m, v in zip(todo, vals):
                self._done[m][x.raw] = v
                a, nxt = self.assign[m], self._next[m]
                f = a.setdefault(f"keccak256_{n}", FuncInterp(0, {}))
                inv = a.setdefault(f"keccak256_{n}-1", FuncInterp(0, {}))
                if (v,) in f.entries:
                    continue
                h = concrete.get((n, v))
                if h is None:
                    k = nxt.get(n, 0) + 1
                    nxt[n] = k
                    lo = km.interval_hook_for_size.get(n, 0) * PART
                    h = (lo + 63) // 64 * 64 + 64 * (k - 1)     # in [lo, lo + PART), % 64 == 0
                f.entries[(v,)] = h
                inv.entries[(h,)] = v
                changed.add(f"keccak256_{n}")
                changed.add(f"keccak256_{n}-1")
        # Power at every symbolic EXP's (base, exponent) under each seed: the
        # exponent manager's axioms for base 256 (Power(256, e) == Power(256,
        # e % 32) and the 256**i table) fix it to 256**(e % 32); any other base
        # takes its true power when positive (the `Power > 0` conjunct), else 1
        sym_pts = exponent_function_manager.symbolic_points
        for j in range(self._sym_pts, len(sym_pts)):
            base, expo = sym_pts[j]
            bs, es = eval_all(base.raw, self.assign), eval_all(expo.raw, self.assign)
            for a, b, e in zip(self.assign, bs, es):
                b, e = int(b), int(e)
                v = 256 ** (e % 32) if b == 256 else pow(b, e, 1 << 256)
                v = v if 0 < v < 1 << 255 else 1
                pw = a["Power"]
                if (b, e) not in pw.entries:
                    pw.entries[(b, e)] = v
                    changed.add("Power")
        self._sym_pts = len(sym_pts)
        for name in changed:
            self._touch(name)

    @property
    def epoch(self):
        return self._epoch

    def models(self) -> List[Model]:
        """The pool, covering every transaction id issued so far.  The Model
        objects keep their identity (the model cache's LRU holds seeds it
        returned): completion only adds entries, so every query a seed answered
        before stays answered."""
        from .transaction import tx_id_manager
        top = int(tx_id_manager._next_transaction_id)
        if top != self._tx_top:
            for k in range(1, top + 1):
                self.add_tx(str(k))
            self._tx_top = top
        from ..smt.exponent_manager import exponent_function_manager
        epoch = (len(self.tx_ids), sum(len(v) for v in self.km.symbolic_inputs.values()),
                 len(self.km.concrete_hashes), len(exponent_function_manager.concrete_points),
                 len(exponent_function_manager.symbolic_points))
        if self._models is None or epoch != self._epoch:
            self._complete()
            if self._models is None:
                self._models = []
                for a in self.assign:
                    ref = ModelRef()
                    ref.assignment = a          # shared: completion updates it in place
                    self._models.append(Model([ref]))
            self._epoch = epoch
        return self._models


def eval_all(raw: Node, assigns: List[Dict[str, object]]) -> List[int]:
    """Value of a bit-vector / Bool term under every assignment (model
    completion: absent variables 0, arrays and functions their default /
    else value), one pass over the DAG with a column of values per node.
    Columns are numpy object arrays of Python ints, so each operator runs as
    one vectorised loop over the models instead of an interpreted call per
    model (the witness completion's hot path)."""
    from ..smt.semantics import apply_op
    n = len(assigns)
    memo: Dict[int, object] = {}

    def col(x):
        out = np.empty(n, dtype=object)
        out[:] = x
        return out

    def arr(node):
        """Per model: (default, {index: value}) of an array term."""
        got = memo.get(id(node))
        if got is not None:
            return got
        if node.op == "array":
            name = node.param[0]
            out = []
            for a in assigns:
                it = a.get(name)
                out.append((it.default, it.entries) if isinstance(it, ArrayInterp) else (0, {}))
        elif node.op == "K":
            d = val(node.args[0])
            out = [(d[m], {}) for m in range(n)]
        elif node.op == "store":
            base, idx, v = arr(node.args[0]), val(node.args[1]), val(node.args[2])
            out = [(base[m][0], {**base[m][1], idx[m]: v[m]}) for m in range(n)]
        else:
            raise ValueError(f"array term {node.op}")
        memo[id(node)] = out
        return out

    def dense_rows(node):
        """Per model (bytes, default) of an `array` term when every model holds
        it as untouched dense bytes, else None."""
        key = ("dense", id(node))
        if key in memo:
            return memo[key]
        rows = None
        if node.op == "array":
            rows = []
            for a in assigns:
                it = a.get(node.param[0])
                raw = it.untouched_dense() if isinstance(it, ArrayInterp) else None
                if raw is None:
                    rows = None
                    break
                rows.append((raw, it.default))
        memo[key] = rows
        return rows

    def cd_word(node):
        """A calldata word (SymbolicCalldata.get_word_at, marked MG_SYM_CDLOAD):
        byte k = If(off + k < size, calldata[off + k], 0) (calldata.py:253-262),
        read straight from each model's calldata bytes -- the 32 ite / select /
        compare columns it would otherwise take.  None when the term is not of
        that shape or a model does not hold the array as bytes."""
        from .symbolic import _PROV, MG_SYM_CDLOAD
        prov = _PROV.get(node)
        if prov is None or prov[0] != MG_SYM_CDLOAD or node.width != 256:
            return None
        first = node
        while first.op == "concat":
            first = first.args[0]
        if first.op != "ite" or first.args[1].op != "select" or first.args[0].op != "bvslt":
            return None
        sel, cond = first.args[1], first.args[0]
        off = prov[2][0].raw
        if sel.args[1] is not off or cond.args[0] is not off or sel.args[0].op != "array":
            return None
        rows = dense_rows(sel.args[0])
        if rows is None:
            return None
        offs, sizes = val(off), val(cond.args[1])
        H, M256 = 1 << 255, (1 << 256) - 1
        out = []
        for (raw, d), o, sz in zip(rows, offs, sizes):
            n_raw = len(raw)
            if o + 32 <= n_raw and o + 31 < sz < H:
                out.append(int.from_bytes(raw[o:o + 32], "big"))
                continue
            ssz = sz - (1 << 256) if sz >= H else sz
            word = 0
            for k in range(32):
                idx = (o + k) & M256
                sidx = idx - (1 << 256) if idx >= H else idx
                byte = (raw[idx] if idx < n_raw else d) if sidx < ssz else 0
                word = (word << 8) | byte
            out.append(word)
        return col(out)

    def signed(x, w):
        return np.where((x >> (w - 1)) & 1, x - (1 << w), x)

    def val(node):
        got = memo.get(id(node))
        if got is not None:
            return got
        op, w = node.op, node.width
        M = (1 << w) - 1 if w else 0
        if op == "concat" and (out := cd_word(node)) is not None:
            pass
        elif op == "const":
            out = col(node.param)
        elif op == "var":
            out = col([(a.get(node.param, 0) if isinstance(a.get(node.param, 0), int) else 0) for a in assigns])
        elif op == "select" and dense_rows(node.args[0]) is not None:
            # a read of an array every model holds as dense bytes (the seeds'
            # calldata): read from the bytes, no entry dicts built
            rows, idx = dense_rows(node.args[0]), val(node.args[1])
            out = col([raw[k] if k < len(raw) else d for (raw, d), k in zip(rows, idx)])
        elif op == "select":
            ar, idx = arr(node.args[0]), val(node.args[1])
            out = col([ar[m][1].get(idx[m], ar[m][0]) for m in range(n)])
        elif op == "uf":
            args = [val(x) for x in node.args]
            name = node.param[0]
            vals = []
            for m, a in enumerate(assigns):
                it = a.get(name)
                key = tuple(c[m] for c in args)
                vals.append(it.entries.get(key, it.else_value) if isinstance(it, FuncInterp) else 0)
            out = col(vals)
        else:
            args = [val(x) for x in node.args]
            ws = [x.width for x in node.args]
            a = args[0] if args else None
            b = args[1] if len(args) > 1 else None
            if op == "bvadd":
                out = (a + b) & M
            elif op == "bvsub":
                out = (a - b) & M
            elif op == "bvmul":
                out = (a * b) & M
            elif op == "bvand":
                out = a & b
            elif op == "bvor":
                out = a | b
            elif op == "bvxor":
                out = a ^ b
            elif op == "bvnot":
                out = ~a & M
            elif op == "bvneg":
                out = -a & M
            elif op in ("eq", "distinct", "bvult", "bvule", "bvugt", "bvuge"):
                cmp = {"eq": np.equal, "distinct": np.not_equal, "bvult": np.less, "bvule": np.less_equal,
                       "bvugt": np.greater, "bvuge": np.greater_equal}[op]
                out = cmp(a, b).astype(np.int64).astype(object)
            elif op in ("bvslt", "bvsle", "bvsgt", "bvsge"):
                cmp = {"bvslt": np.less, "bvsle": np.less_equal, "bvsgt": np.greater,
                       "bvsge": np.greater_equal}[op]
                out = cmp(signed(a, ws[0]), signed(b, ws[0])).astype(np.int64).astype(object)
            elif op == "not":
                out = (a & 1) ^ 1
            elif op == "and":
                out = col(1)
                for c in args:
                    out = out & (c & 1)
            elif op == "or":
                out = col(0)
                for c in args:
                    out = out | (c & 1)
            elif op == "ite":
                out = np.where((a & 1).astype(bool), args[1], args[2])
            elif op == "concat":
                out = (a << ws[1]) | b
            elif op == "extract":
                out = (a >> node.param[1]) & M
            elif op == "zero_extend":
                out = a
            else:                               # the rest one model at a time
                out = col([apply_op(op, w, [c[m] for c in args], ws, node.param) for m in range(n)])
        memo[id(node)] = out
        return out

    return list(val(raw))
