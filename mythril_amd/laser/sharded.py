"""Multi-transaction runs with the open world states sharded over the ranks
(SURVEY §8(e), config C5).

The reference's transaction loop (svm.py:239-275 ``_execute_transactions``)
starts one transaction per open world state, runs ``exec()`` and collects the
surviving world states as the next transaction's ``open_states``.  Here a
transaction round is one concrete ``MessageCallTransaction`` per (open world
state, calldata) pair — the symbolic calldata of the reference sampled by a
list of concrete calldatas — and the pairs of a round are partitioned over the
ranks, one process per GPU:

* the first round deals the (replicated) initial pairs round-robin, pair g to
  rank g % world; from then on every rank keeps the world states its own
  paths produced (no state ever crosses ranks — no data-path collective);
* the pairs a rank starts all run as lanes of ONE ``exec()``, i.e. one kernel-1
  batch per round per GPU;
* per round, the only exchange is a small all-gather: every rank's pair count
  (so transaction ids are the global pair positions, in rank-major order, and
  every rank's id counter advances by the global count — the re-sync §8(e)
  asks for, transaction_models.py:21-36) and the coverage bytes of every code
  (OR, coverage_plugin.py semantics) over RCCL (``dist.allgather_coverage``).

With one rank this is exactly the single-process loop.  The union over ranks
of the open world states equals the single-process run's (as a multiset of
account states; only the transaction ids differ, as §8(e) allows).
"""
from __future__ import annotations

from copy import copy
from typing import Dict, List, Optional, Sequence

import struct

import numpy as np

from .disassembly import Disassembly
from .transaction import MessageCallTransaction, _setup_global_state_for_execution, tx_id_manager


def _allgather_ints(x: int) -> List[int]:
    from .. import dist as mdist
    rank, world = mdist.rank_world()
    if world == 1:
        return [int(x)]
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(x)], dtype=torch.int64, device=mdist._device())
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def _allgather_keys(keys: Sequence[str]) -> List[str]:
    from .. import dist as mdist
    rank, world = mdist.rank_world()
    if world == 1:
        return sorted(keys)
    return sorted(set(k for part in _allgather_values(sorted(keys)) for k in part))


def exchange_coverage(laser_evm) -> Dict[str, np.ndarray]:
    """OR of every rank's coverage table ({bytecode: bytes}) into this rank's
    LaserEVM (it then reports the union, as one process covering every shard
    would); returns the union."""
    from .. import dist as mdist
    local = {code: np.asarray(bits, dtype=np.uint8) for code, (_, bits) in
             laser_evm.coverage().items()}
    union: Dict[str, np.ndarray] = {}
    for code in _allgather_keys(list(local)):
        n = _allgather_ints(local[code].size if code in local else 0)
        mine = np.zeros(max(n), dtype=np.uint8)
        if code in local:
            mine[:local[code].size] = local[code]
        union[code] = mdist.allgather_coverage(mine)
    laser_evm.merge_peer_coverage(union)
    return union


# ---------------------------------------------------------------- models over a tensor
# A model travels as a stream of u32 words (no pickled objects): the stream of
# every rank rides one RCCL all-gather (dist.allgather_models, [k, 1, 8] rows).
#   stream  := n_models model*
#   model   := n_refs ref*
#   ref     := n_items item*
#   item    := name kind (int: big | array: big(default) n (big big)* |
#                         func: big(else) n (n_args big* big)*)
#   name    := n_bytes word*   (utf-8, zero padded)
#   big     := n_limbs limb*   (little-endian u32 limbs)
def _put_big(out: list, v: int) -> None:
    v = int(v)
    limbs = []
    while v:
        limbs.append(v & 0xFFFFFFFF)
        v >>= 32
    out.append(len(limbs))
    out.extend(limbs)


def _put_name(out: list, name: str) -> None:
    b = name.encode()
    out.append(len(b))
    b = b + b"\0" * (-len(b) % 4)
    out.extend(int.from_bytes(b[k:k + 4], "little") for k in range(0, len(b), 4))


def _models_to_words(models) -> np.ndarray:
    from ..smt.program import ArrayInterp, FuncInterp
    out = [len(models)]
    for m in models:
        refs = getattr(m, "raw", [m])
        out.append(len(refs))
        for ref in refs:
            items = list(ref.assignment.items())
            out.append(len(items))
            for name, v in items:
                _put_name(out, name)
                if isinstance(v, ArrayInterp):
                    out.append(1)
                    _put_big(out, v.default)
                    out.append(len(v.entries))
                    for k, x in v.entries.items():
                        _put_big(out, k)
                        _put_big(out, x)
                elif isinstance(v, FuncInterp):
                    out.append(2)
                    _put_big(out, v.else_value)
                    out.append(len(v.entries))
                    for args, x in v.entries.items():
                        out.append(len(args))
                        for a in args:
                            _put_big(out, a)
                        _put_big(out, x)
                else:
                    out.append(0)
                    _put_big(out, v)
    return np.asarray(out, dtype=np.uint32)


class _Words:
    def __init__(self, w):
        self.w, self.k = w, 0

    def u(self) -> int:
        x = int(self.w[self.k])
        self.k += 1
        return x

    def big(self) -> int:
        n = self.u()
        v = 0
        for j in range(n):
            v |= int(self.w[self.k + j]) << (32 * j)
        self.k += n
        return v

    def name(self) -> str:
        n = self.u()
        nw = (n + 3) // 4
        b = b"".join(int(x).to_bytes(4, "little") for x in self.w[self.k:self.k + nw])
        self.k += nw
        return b[:n].decode()


# ---------------------------------------------------------------- values over a tensor
# Plain values (None, bool, int of any size and sign, str, bytes, tuple, list,
# dict) as a u32 stream: a tag word, then the payload; what travels between
# ranks besides models (code keys, keccak / EXP registrations, issues).
_T_NONE, _T_FALSE, _T_TRUE, _T_INT, _T_NEG, _T_STR, _T_BYTES, _T_TUPLE, _T_LIST, _T_DICT, _T_FLOAT = range(11)


def _put_bytes(out: list, b: bytes) -> None:
    out.append(len(b))
    b = b + b"\0" * (-len(b) % 4)
    out.extend(int.from_bytes(b[k:k + 4], "little") for k in range(0, len(b), 4))


def _put_value(out: list, v) -> None:
    if v is None:
        out.append(_T_NONE)
    elif v is True or v is False:
        out.append(_T_TRUE if v else _T_FALSE)
    elif isinstance(v, int):
        out.append(_T_INT if v >= 0 else _T_NEG)
        _put_big(out, abs(v))
    elif isinstance(v, float):
        out.append(_T_FLOAT)                    # IEEE-754 binary64, two words
        _put_bytes(out, struct.pack("<d", v))
    elif isinstance(v, str):
        out.append(_T_STR)
        _put_bytes(out, v.encode())
    elif isinstance(v, (bytes, bytearray)):
        out.append(_T_BYTES)
        _put_bytes(out, bytes(v))
    elif isinstance(v, (tuple, list)):
        out.append(_T_TUPLE if isinstance(v, tuple) else _T_LIST)
        out.append(len(v))
        for x in v:
            _put_value(out, x)
    elif isinstance(v, dict):
        out.append(_T_DICT)
        out.append(len(v))
        for k, x in v.items():
            _put_value(out, k)
            _put_value(out, x)
    else:
        raise TypeError(f"cannot send a {type(v).__name__} between ranks")


def _values_to_words(v) -> np.ndarray:
    out: list = []
    _put_value(out, v)
    return np.asarray(out, dtype=np.uint32)


def _get_bytes(r: "_Words") -> bytes:
    n = r.u()
    nw = (n + 3) // 4
    b = b"".join(int(x).to_bytes(4, "little") for x in r.w[r.k:r.k + nw])
    r.k += nw
    return b[:n]


def _get_value(r: "_Words"):
    t = r.u()
    if t == _T_NONE:
        return None
    if t in (_T_FALSE, _T_TRUE):
        return t == _T_TRUE
    if t in (_T_INT, _T_NEG):
        v = r.big()
        return v if t == _T_INT else -v
    if t == _T_FLOAT:
        return struct.unpack("<d", _get_bytes(r))[0]
    if t == _T_STR:
        return _get_bytes(r).decode()
    if t == _T_BYTES:
        return _get_bytes(r)
    if t in (_T_TUPLE, _T_LIST):
        xs = [_get_value(r) for _ in range(r.u())]
        return tuple(xs) if t == _T_TUPLE else xs
    if t == _T_DICT:
        d = {}
        for _ in range(r.u()):
            k = _get_value(r)
            d[k] = _get_value(r)
        return d
    raise ValueError(f"bad value tag {t}")


def _allgather_values(v) -> list:
    """Every rank's value (rank order) through one u32 tensor all-gather."""
    from .. import dist as mdist
    _, world = mdist.rank_world()
    if world == 1:
        return [v]
    return [_get_value(_Words(w)) if w.size else None for w in _allgather_words(_values_to_words(v))]


def _words_to_models(words: np.ndarray) -> list:
    from ..smt.program import ArrayInterp, FuncInterp
    from ..smt.solver import Model, ModelRef
    r = _Words(words)
    models = []
    for _ in range(r.u()):
        refs = []
        for _ in range(r.u()):
            d = {}
            for _ in range(r.u()):
                name, kind = r.name(), r.u()
                if kind == 1:
                    dflt = r.big()
                    d[name] = ArrayInterp(dflt, {r.big(): r.big() for _ in range(r.u())})
                elif kind == 2:
                    els = r.big()
                    ent = {}
                    for _ in range(r.u()):
                        args = tuple(r.big() for _ in range(r.u()))
                        ent[args] = r.big()
                    d[name] = FuncInterp(els, ent)
                else:
                    d[name] = r.big()
            refs.append(ModelRef(d))
        models.append(Model(refs))
    return models


def _allgather_words(words: np.ndarray) -> List[np.ndarray]:
    """Every rank's u32 stream (rank order) through one tensor all-gather."""
    from .. import dist as mdist
    rank, world = mdist.rank_world()
    n = int(words.size)
    rows = np.zeros(((n + 1 + 7) // 8, 1, 8), dtype=np.uint32)
    flat = rows.reshape(-1)
    flat[0] = n
    flat[1:n + 1] = words
    got = mdist.allgather_models(rows)
    counts = _allgather_ints(rows.shape[0])
    out, at = [], 0
    for c in counts:
        f = got[at:at + c].reshape(-1)
        out.append(f[1:1 + int(f[0])] if c else np.zeros(0, dtype=np.uint32))
        at += c
    return out


def exchange_models(model_cache=None) -> int:
    """the satisfying models every rank found since the last
    exchange (backend answers cached by get_model, support/model.py:76-78)
    join every other rank's candidate pool -- kernel 2's ModelCache -- in rank
    order, each with count 1 as a fresh backend model gets.  The models ride a
    u32 tensor all-gather (dist.allgather_models), one per transaction round;
    returns the number of peer models received."""
    from .. import dist as mdist
    from ..smt import solver
    cache = model_cache or solver.model_cache
    rank, world = mdist.rank_world()
    mine = _models_to_words(cache.take_fresh())
    if world == 1:
        return 0
    got = 0
    for r, words in enumerate(_allgather_words(mine)):
        if r == rank or words.size == 0:
            continue
        for m in _words_to_models(words):
            cache.put(m, 1, peer=True)
            got += 1
    return got


def execute_message_calls(laser_evm, callee_address, caller_address, origin_address,
                          datas: Sequence[bytes], gas_limit, gas_price, value, code=None,
                          track_gas: bool = False, exchange_cov: bool = True):
    """One transaction round: a MessageCallTransaction for every (open world
    state, calldata) pair this rank owns, all run by one ``laser_evm.exec``.
    Returns the final states when ``track_gas`` (this rank's paths)."""
    from .. import dist as mdist
    rank, world = mdist.rank_world()
    open_states = laser_evm.open_states[:]
    del laser_evm.open_states[:]
    if getattr(laser_evm, "use_reachability_check", False):
        # svm.py:244-249: a transaction starts only from open states whose path
        # constraints are possible (kernel-2 quick-sat, then the SMT backend)
        from ..smt.solver import Constraints
        open_states = [ws for ws in open_states if Constraints(ws.constraints).is_possible()]
    local = [(ws, d) for ws in open_states for d in datas]
    if world > 1 and not getattr(laser_evm, "_sharded", False):
        # replicated start: deal pair g to rank g % world
        total = len(local)
        mine = [(g, p) for g, p in enumerate(local) if g % world == rank]
    else:
        counts = _allgather_ints(len(local))
        off = sum(counts[:rank])
        total = sum(counts)
        mine = [(off + j, p) for j, p in enumerate(local)]
    base = tx_id_manager._next_transaction_id
    for g, (ws, data) in mine:
        # every calldata of a world state starts from its own copy of it
        world_state = ws if len(datas) == 1 else copy(ws)
        bytecode = code or world_state[callee_address].code.bytecode
        tx = MessageCallTransaction(
            world_state=world_state,
            identifier=str(base + g + 1),
            gas_price=gas_price,
            gas_limit=gas_limit,
            origin=origin_address,
            code=Disassembly(bytecode),
            caller=caller_address,
            callee_account=world_state[callee_address],
            call_data=data,
            call_value=value,
        )
        _setup_global_state_for_execution(laser_evm, tx)
    tx_id_manager.set_counter(base + total)
    laser_evm._sharded = world > 1
    final = laser_evm.exec(track_gas=track_gas)
    if exchange_cov and world > 1 and laser_evm.record_coverage:
        exchange_coverage(laser_evm)
    if world > 1:
        exchange_models()
    return final


def open_state_counts(laser_evm) -> List[int]:
    """Every rank's number of open world states (rank order)."""
    return _allgather_ints(len(laser_evm.open_states))


# ---------------------------------------------------------------- world states across ranks
class _NodeTable:
    """Expression DAG nodes as a flat post-order table (op, width, arg indices,
    param): shared subterms once, no recursion, re-interned on load (Node is
    hash-consed, so a received term IS the local term wherever both exist)."""

    def __init__(self):
        self.rows: List[tuple] = []
        self.index: Dict[int, int] = {}
        self._keep: List = []

    def add(self, node) -> int:
        got = self.index.get(id(node))
        if got is not None:
            return got
        stack = [(node, False)]
        while stack:
            n, done = stack.pop()
            if id(n) in self.index:
                continue
            if not done:
                stack.append((n, True))
                stack.extend((a, False) for a in n.args if id(a) not in self.index)
                continue
            self.index[id(n)] = len(self.rows)
            self._keep.append(n)
            self.rows.append((n.op, n.width, tuple(self.index[id(a)] for a in n.args), n.param))
        return self.index[id(node)]

    @staticmethod
    def load(rows) -> list:
        from ..smt.expr import Node
        out: list = []
        for op, width, args, param in rows:
            out.append(Node(op, width, tuple(out[a] for a in args), param))
        return out


def _dumps_states(items, shared: Dict[int, int]) -> bytes:
    """Pickle [(position, world state)] with expression nodes as table rows and
    rank-global objects (detection modules, the LaserEVM) as references."""
    import io
    import pickle
    from ..smt.expr import Node
    table = _NodeTable()

    class P(pickle.Pickler):
        def persistent_id(self, obj):
            if type(obj) is Node:
                return ("N", table.add(obj))
            k = shared.get(id(obj))
            return None if k is None else ("S", k)

    buf = io.BytesIO()
    P(buf, protocol=pickle.HIGHEST_PROTOCOL).dump(items)
    return pickle.dumps((table.rows, buf.getvalue()), protocol=pickle.HIGHEST_PROTOCOL)


def _loads_states(blob: bytes, shared_objs: list):
    import io
    import pickle
    rows, payload = pickle.loads(blob)
    nodes = _NodeTable.load(rows)

    class U(pickle.Unpickler):
        def persistent_load(self, pid):
            kind, k = pid
            return nodes[k] if kind == "N" else shared_objs[k]

    return U(io.BytesIO(payload)).load()


def _shared_objects(laser_evm) -> list:
    """Objects every rank holds once and states only refer to: the LaserEVM and
    the detection modules whose hooks it runs (an IssueAnnotation's detector)."""
    objs, seen = [laser_evm], {id(laser_evm)}
    for table in (getattr(laser_evm, "pre_hooks", {}), getattr(laser_evm, "post_hooks", {})):
        for hooks in table.values():
            for h in hooks:
                m = getattr(h, "__self__", None)
                if m is not None and id(m) not in seen:
                    seen.add(id(m))
                    objs.append(m)
    return objs


def rebalance(laser_evm) -> List[int]:
    """SURVEY §8(e) rebalancing at a transaction boundary: the open world
    states of all ranks, in rank-major order, are re-dealt in equal contiguous
    runs (rank r gets positions [t_r, t_r + n_r), n_r = total // world, the
    first total % world ranks one more).  Only states that change owner move,
    each straight to its new owner (one all-to-all of pickled states, dist.
    alltoall_bytes; expression nodes as flat tables).
    Returns the per-rank counts before the move."""
    from .. import dist as mdist
    rank, world = mdist.rank_world()
    counts = _allgather_ints(len(laser_evm.open_states))
    if world == 1:
        return counts
    total = sum(counts)
    target = [total // world + (1 if r < total % world else 0) for r in range(world)]
    tstart = [sum(target[:r]) for r in range(world)]
    off = sum(counts[:rank])

    def owner(g):
        for q in range(world):
            if g < tstart[q] + target[q]:
                return q
        return world - 1

    keep, send = [], {}
    for j, ws in enumerate(laser_evm.open_states):
        g = off + j
        q = owner(g)
        (keep if q == rank else send.setdefault(q, [])).append((g, ws))
    objs = _shared_objects(laser_evm)
    shared = {id(o): k for k, o in enumerate(objs)}
    # one payload per destination, exchanged point to point (an all-to-all):
    # a state crosses the fabric once, to the rank that takes it over
    blobs = [_dumps_states({q: send[q]}, shared) if send.get(q) else b"" for q in range(world)]
    parts = mdist.alltoall_bytes(blobs)
    got = list(keep)
    for r, b in enumerate(parts):
        if r == rank or not b:
            continue
        got.extend(_loads_states(b, objs).get(rank, []))
    got.sort(key=lambda x: x[0])
    laser_evm.open_states = [ws for _, ws in got]
    return counts


def sync_function_managers() -> int:
    """Every rank registers the keccak inputs (symbolic and concrete) and the
    concrete EXP points the other ranks registered, so the axioms
    create_conditions adds cover every term a (moved) state's constraints
    mention (keccak_function_manager.py:116-179, exponent_function_manager.py:
    32-60).  Returns the number of entries received."""
    from .. import dist as mdist
    from ..smt.exponent_manager import exponent_function_manager as em
    from ..smt.expr import BitVec
    from ..smt.keccak_manager import keccak_function_manager as km
    rank, world = mdist.rank_world()
    if world == 1:
        return 0
    table = _NodeTable()
    sym = [table.add(x.raw) for xs in km.symbolic_inputs.values() for x in xs]
    conc = [(table.add(k.raw), table.add(h.raw)) for k, h in km.concrete_hashes.items()]
    pts = sorted(em.concrete_points.items())
    # node rows (op, width, args, param) and indices as a u32 value stream (no pickling)
    parts = _allgather_values((table.rows, sym, conc, pts))
    have = {id(x.raw) for xs in km.symbolic_inputs.values() for x in xs}
    have_c = {id(k.raw) for k in km.concrete_hashes}
    got = 0
    for r, part in enumerate(parts):
        if r == rank or not part:
            continue
        rows, s_idx, c_idx, p = part
        nodes = _NodeTable.load(rows)
        for i in s_idx:
            n = nodes[i]
            if id(n) not in have:
                have.add(id(n))
                km.get_function(n.width)
                x = BitVec(n)
                func, _ = km.get_function(n.width)
                km.symbolic_inputs.setdefault(n.width, []).append(x)
                km.hash_result_store[n.width].append(func(x))
                got += 1
        for ki, hi in c_idx:
            k = nodes[ki]
            if id(k) not in have_c:
                have_c.add(id(k))
                km.get_function(k.width)
                km.concrete_hashes[BitVec(k)] = BitVec(nodes[hi])
                got += 1
        for key, v in p:
            if tuple(key) not in em.concrete_points:
                em.concrete_points[tuple(key)] = v
                got += 1
    return got


def _issue_code_key(d: dict):
    """The code half of a module's cache key for an issue's attribute dict:
    the reference's Issue stores bytecode_hash (report.py:70) and the modules
    cache (address, bytecode_hash) (base.py:63-70, exceptions.py:57); an issue
    type that keeps the bytecode itself is keyed on that."""
    if d.get("bytecode_hash") is not None:
        return d["bytecode_hash"]
    return d.get("bytecode")


def merge_issues(modules, issue_type=None) -> int:
    """after sharded rounds every rank holds the issues its own
    paths filed.  All ranks' issues of each detection module (same module
    order on every rank) are gathered in rank order and de-duplicated by the
    modules' own cache key -- (address, code hash) for the modules that cache
    automatically (base.py:63-96), (source location, code hash) for
    Exceptions -- keeping the first; each module's ``issues`` become the
    merged set on every rank and its cache gets their keys through the
    module's own ``update_cache`` (or, for a module that caches by source
    location, in that form), so re-detection is suppressed as the module
    itself would suppress it.  Issues travel as their attribute dicts (value
    stream, no pickling; floats such as discovery_time included) and are
    rebuilt as `issue_type` (default: the class of the issues the local
    modules hold).  An attribute the stream cannot carry raises TypeError
    rather than being dropped.  Returns the merged count."""
    from .. import dist as mdist
    _, world = mdist.rank_world()
    local = []
    for m in modules:
        rows = []
        for i in m.issues:
            d = dict(vars(i))
            for k, v in d.items():
                if not _sendable(v):
                    raise TypeError(f"issue attribute {k!r} ({type(v).__name__}) cannot be sent between ranks")
            rows.append(d)
        local.append(rows)
    parts = _allgather_values(local) if world > 1 else [local]
    cls = issue_type or next((type(i) for m in modules for i in m.issues), None)
    total = 0
    for k, m in enumerate(modules):
        by_location = getattr(m, "auto_cache", True) is False
        merged, keys = [], set()
        for part in parts:
            for d in (part[k] if part else []):
                key = (d.get("source_location") if by_location else d.get("address"), _issue_code_key(d))
                if key in keys:
                    continue
                keys.add(key)
                issue = object.__new__(cls) if cls is not None else _Issue()
                issue.__dict__.update(d)
                merged.append(issue)
        m.issues = merged
        if by_location or not hasattr(m, "update_cache"):
            m.cache |= keys
        else:
            m.update_cache(merged)
        total += len(merged)
    return total


class _Issue:
    """A received issue when no local module holds one of the report's class."""


def _sendable(v) -> bool:
    try:
        _values_to_words(v)
        return True
    except TypeError:
        return False


def execute_symbolic_transactions(laser_evm, callee_address, tx_count: Optional[int] = None,
                                  gas_limit: int = 8_000_000, balance: bool = True) -> None:
    """svm.py:230-275 ``_execute_transactions`` with the open states sharded
    over the ranks: per transaction round, the states are
    rebalanced (``rebalance``), filtered for reachability, and each rank runs
    one symbolic message call per state it owns -- one ``exec()``, its lanes on
    this rank's GPU.  Transaction ids are the global positions (rank-major),
    so every rank's counter advances by the global count (transaction_models.py
    :21-36); after the round the function managers, coverage and fresh models
    are exchanged.  With one rank this is exactly the single-process loop.
    The first round deals a replicated start round-robin."""
    from .. import dist as mdist
    from .transaction import execute_symbolic_message_call
    from datetime import datetime
    rank, world = mdist.rank_world()
    n = laser_evm.transaction_count if tx_count is None else tx_count
    for hook in laser_evm._start_exec_trans_hooks:       # svm.py:214-228 execute_transactions
        hook()
    laser_evm.time = datetime.now()
    if world > 1 and not getattr(laser_evm, "_sharded", False):
        laser_evm.open_states = mdist.shard(laser_evm.open_states, rank, world)
        laser_evm._sharded = True
    for _ in range(n):
        if balance:
            rebalance(laser_evm)
        if laser_evm.use_reachability_check:
            laser_evm.open_states = laser_evm.reachable(laser_evm.open_states)
        counts = _allgather_ints(len(laser_evm.open_states))
        if sum(counts) == 0:
            break
        base = tx_id_manager._next_transaction_id
        off = sum(counts[:rank])
        ids = [str(base + off + j + 1) for j in range(counts[rank])]
        # the counter covers the round's ids before the calls run, as the
        # reference's get_next_tx_id per call leaves it (witness seeds and the
        # solver read it while the transactions execute)
        tx_id_manager.set_counter(base + sum(counts))
        for hook in laser_evm._start_sym_trans_hooks:
            hook()
        execute_symbolic_message_call(laser_evm, callee_address, gas_limit, ids=ids)
        for hook in laser_evm._stop_sym_trans_hooks:
            hook()
        if world > 1:
            sync_function_managers()
            if laser_evm.record_coverage:
                exchange_coverage(laser_evm)
            exchange_models()
    laser_evm.executed_transactions = True
    for hook in laser_evm._stop_exec_trans_hooks:
        hook()
