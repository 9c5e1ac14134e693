"""Symbolic lanes: the host half of the expression arena.

A symbolic lane (MG_LANE_SYMBOLIC) keeps, next to every stack word, a tag: 0 for
a concrete value, else 1 + the index of the arena node that defines it
(include/mythgpu.h, mythril_amd/csrc/sym_step.cuh).  This module turns arena
nodes into the expressions the reference's mutators build for the same
instruction sequence, and back:

* sources: ``SymbolicCalldata.get_word_at`` / ``calldatasize``
  (state/calldata.py:214-262, with its signed ``item < size`` bound check) and
  the symbolic environment words of a symbolic transaction (``sender_{id}``,
  ``call_value{id}``, ``gas_price{id}``, transaction/symbolic.py:105-150);
* ALU nodes: the reference's construction rules (instructions.py:356-760):
  ``pop_bitvec`` turns a Bool operand into ``If(b, 1, 0)``; LT/GT/SLT/SGT/EQ
  push Bools; ISZERO pushes ``If(Not(b) | v == 0, 1, 0)``; NOT is
  ``2**256 - 1 - v``; DIV/SDIV/MOD/SMOD are UDiv / signed div / URem / SRem;
  SHL/SHR/SAR are ``<<``, LShR, ``>>``; BYTE with a concrete index is
  ``Concat(0_248, Extract(off + 7, off, v))``.  The expression layer folds
  constants as z3's ``simplify`` would; expressions are hash-consed, so equal
  constructions are the same node.

``decode_stack`` builds a lane's stack from its planes, ``encode_stack``
writes an expression stack back (only expressions this module produced, found
through their recorded provenance; anything else raises ``NotEncodable`` and
the state stays with the host's handler).  ``jumpi_successors`` forks a lane
stopped with MG_FORK exactly as instructions.py:1558-1636 does.
"""
from __future__ import annotations

import bisect
import weakref
from copy import copy, deepcopy
from typing import List, Optional, Tuple

import numpy as np

from ..lanes import (ENV_ADDRESS as MG_ENV_ADDRESS, ENV_CALLER as MG_ENV_CALLER,
                     ENV_CALLVALUE as MG_ENV_CALLVALUE, ENV_GASPRICE as MG_ENV_GASPRICE,
                     ENV_ORIGIN as MG_ENV_ORIGIN, MG_LANE_MEMTAG, MG_LANE_SYMBOLIC, MG_LANE_SYMCD,
                     MG_LANE_SYMENV_SHIFT, MG_LANE_SYMSTORE, MG_SYM_BIN, MG_SYM_CDBYTE, MG_SYM_CDBYTEX, MG_SYM_CDLOAD,
                     MG_SYM_MLOADK, MG_SYM_MSTOREK,
                     MG_ENV_CHAINID, MG_ENV_COINBASE, MG_ENV_DIFFICULTY, MG_ENV_GAS, MG_ENV_NUMBER, MG_LANE_SYMBLOCK, MG_ENV_RETURNDATASIZE, MG_ENV_TIMESTAMP, MG_ENV_SELFBALANCE, MG_LANE_SYMBAL, MG_LANE_SYMRDS, MG_SYM_BALANCE, MG_SYM_CDSIZE, MG_SYM_CONCAT, MG_SYM_CONST, MG_SYM_ENV, MG_SYM_EXTRACT, MG_SYM_KECCAK, MG_SYM_SLOAD,
                     MG_SYM_TERM, MG_SYM_UN, limbs_to_word, word_to_limbs)
from ..smt.expr import (Array, BitVec, Bool, Concat, Extract, Function, If, LShR, Node, Not, UDiv, UGT, ULT,
                        URem, SRem, _select, simplify_concat, symbol_factory)
from .state import Memory, Storage

TT256M1 = (1 << 256) - 1


class NotEncodable(Exception):
    """An expression the arena cannot represent (it did not come from a node)."""


class SymbolicCalldata:
    """state/calldata.py:214-262: calldata of a symbolic transaction — an
    ``{id}_calldata`` byte array and a ``{id}_calldatasize`` word."""

    def __init__(self, tx_id: str):
        self.tx_id = str(tx_id)
        self._size = symbol_factory.BitVecSym(f"{tx_id}_calldatasize", 256)
        self._calldata = Array(f"{tx_id}_calldata", 256, 8)
        self._words = {}            # offset node -> word expression (hash-consed anyway)

    @property
    def size(self) -> BitVec:
        return self._size

    @property
    def calldatasize(self) -> BitVec:
        return self._size

    def _load(self, item) -> BitVec:
        item = symbol_factory.BitVecVal(item, 256) if isinstance(item, int) else item
        return If(item < self._size, self._calldata[item], symbol_factory.BitVecVal(0, 8))

    def __getitem__(self, item) -> BitVec:
        """calldata.py:57-64 for an int or expression index: one byte,
        If(index < calldatasize, calldata[index], 0) (calldata.py:253-262)."""
        return self._load(item)

    def get_word_at(self, offset) -> BitVec:
        """BaseCalldata.get_word_at: Concat of the 32 loads at offset + k."""
        off = symbol_factory.BitVecVal(offset, 256) if isinstance(offset, int) else offset
        w = self._words.get(off.raw)
        if w is None:
            w = self._words[off.raw] = _mark(Concat(*[self._load(off if k == 0 else off + k) for k in range(32)]),
                                             MG_SYM_CDLOAD, 0, (off,))
        return w

    def __len__(self):
        return 0


def is_symbolic_calldata(cd) -> bool:
    return isinstance(cd, SymbolicCalldata)


# ----------------------------------------------------------- provenance
# raw node -> (kind, imm, operand expressions): what encode_stack replays
_PROV: "weakref.WeakKeyDictionary[Node, tuple]" = weakref.WeakKeyDictionary()


def _mark(e, kind: int, imm: int, args: tuple, width: int = 256):
    """Record how node `e` was built.  A Bool result goes on the stack as
    If(b, 1, 0), as MachineStack.append wraps it (machine_state.py:39-46); the
    wrapper is what the stack holds and what encode_stack maps back to the
    (width-1) node."""
    if isinstance(e, Bool):
        e = If(e, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
        width = 1
    try:
        _PROV[e.raw] = (kind, imm, args, width)
    except TypeError:
        pass
    return e


def as_bitvec(x) -> BitVec:
    """util.pop_bitvec (util.py:75-96)."""
    if isinstance(x, Bool):
        return If(x, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
    return x


_ENV_ATTR = {MG_ENV_ADDRESS: "address", MG_ENV_CALLER: "sender", MG_ENV_ORIGIN: "origin",
             MG_ENV_CALLVALUE: "callvalue", MG_ENV_GASPRICE: "gasprice"}


def binary(op: int, a, b):
    """The reference's expression for binary opcode `op` on (first pop a, second pop b)."""
    if op in (0x01, 0x02, 0x03):
        x, y = as_bitvec(a), as_bitvec(b)
        return x + y if op == 0x01 else x * y if op == 0x02 else x - y
    if op in (0x04, 0x05, 0x06, 0x07):                      # device: divisor is not a concrete 0
        x, y = as_bitvec(a), as_bitvec(b)
        return {0x04: UDiv, 0x05: lambda p, q: p / q, 0x06: URem, 0x07: SRem}[op](x, y)
    if op == 0x10:
        return ULT(as_bitvec(a), as_bitvec(b))
    if op == 0x11:
        return UGT(as_bitvec(a), as_bitvec(b))
    if op == 0x12:
        return as_bitvec(a) < as_bitvec(b)
    if op == 0x13:
        return as_bitvec(a) > as_bitvec(b)
    if op == 0x14:
        return as_bitvec(a) == as_bitvec(b)
    if op in (0x16, 0x17):
        x, y = as_bitvec(a), as_bitvec(b)
        return x & y if op == 0x16 else x | y
    if op == 0x18:
        return a ^ b
    if op == 0x1A:                                          # a = concrete index < 32
        off = (31 - int(a.value)) * 8
        return Concat(symbol_factory.BitVecVal(0, 248), Extract(off + 7, off, b))
    if op == 0x1B:
        return as_bitvec(b) << as_bitvec(a)
    if op == 0x1C:
        return LShR(as_bitvec(b), as_bitvec(a))
    if op == 0x1D:
        return as_bitvec(b) >> as_bitvec(a)
    if op == 0x0A:                                          # EXP: Power(base, exponent)
        from ..smt.exponent_manager import exponent_function_manager
        return exponent_function_manager.create_condition(as_bitvec(a), as_bitvec(b))[0]
    raise NotEncodable(f"no symbolic semantics for opcode {op:#x}")


def unary(op: int, a):
    if op == 0x15:                                           # ISZERO
        exp = Not(a) if isinstance(a, Bool) else a == 0
        return If(exp, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
    if op == 0x19:                                           # NOT: TT256M1 - x
        return symbol_factory.BitVecVal(TT256M1, 256) - a
    raise NotEncodable(f"no symbolic semantics for opcode {op:#x}")


# the opcodes that push the transaction's fresh variable of a name (instructions.py:
# 1386-1425, 1700-1709): MG_SYM_ENV immediates
_FRESH = {MG_ENV_GAS: "gas", MG_ENV_COINBASE: "coinbase", MG_ENV_TIMESTAMP: "timestamp",
          MG_ENV_DIFFICULTY: "block_difficulty"}


def source(kind: int, imm: int, arg, state):
    env = state.environment
    if kind == MG_SYM_CDLOAD:
        return env.calldata.get_word_at(arg)
    if kind == MG_SYM_CDSIZE:
        return env.calldata.calldatasize
    if kind == MG_SYM_ENV:
        if imm == MG_ENV_SELFBALANCE:           # selfbalance_ (instructions.py:968-976)
            return env.active_account.balance()
        if imm == MG_ENV_RETURNDATASIZE:        # returndatasize_ (instructions.py:1359-1370)
            return state.last_return_data.size
        if imm in _FRESH:                       # gas_, coinbase_, timestamp_, difficulty_
            return state.new_bitvec(_FRESH[imm], 256)
        if imm == MG_ENV_NUMBER:                # number_ (instructions.py:1406-1413)
            return env.block_number
        if imm == MG_ENV_CHAINID:               # chainid_ (instructions.py:958-965)
            return env.chainid
        return getattr(env, _ENV_ATTR[imm])
    raise NotEncodable(f"unknown source kind {kind}")


def balance_of(state, address):
    """balance_ (instructions.py:907-931) with no dynamic loader: a known concrete
    address gives its account's balance(); otherwise (symbolic, or a concrete
    address accounts_exist_or_load cannot load) the If chain over the world
    state's accounts, in their order."""
    ws = state.world_state
    v = address.value
    if v is not None and v in ws.accounts:
        return ws.accounts[v].balance()
    bal = symbol_factory.BitVecVal(0, 256)
    for a in ws.accounts.values():
        bal = If(address == a.address, a.balance(), bal)
    return bal


# ----------------------------------------------------------- decode / encode
class _Decoder:
    """The expressions of one lane's planes: its stack words, memory bytes and
    storage chain (the arena is shared by all three, nodes memoised)."""

    def __init__(self, b, i: int, state, prefix: Optional[list] = None):
        self.b, self.i, self.state = b, i, state
        self.n_nodes = int(b.n_nodes[i])
        self.memo: List[Optional[object]] = [None] * self.n_nodes
        # the terms of the nodes the host encoded into this lane (the arena only
        # grows on the device): node k < len(prefix) decodes to prefix[k] with no
        # rebuild of its expression
        self.prefix = prefix if prefix is not None and len(prefix) <= self.n_nodes else None
        self._rows = None
        self._entries = None
        self._raws = None

    def row(self, k: int):
        """Node k's (x, y, z, w) as ints (the lane's node rows read once)."""
        if self._rows is None:
            self._rows = self.b.node[self.i, :self.n_nodes].tolist()
        return self._rows[k]

    # -- operands
    def const(self, r: int, width: int = 256):
        v = limbs_to_word(self.b.cval[self.i, r & ~MG_SYM_CONST])
        return symbol_factory.BitVecVal(v & ((1 << width) - 1), width)

    def ref(self, r: int):
        return self.const(r) if r & MG_SYM_CONST else self.node(r)

    def parts(self, r: int, width: int) -> list:
        """The memory parts an operand of a CONCAT / KECCAK stands for."""
        if r & MG_SYM_CONST:
            return [self.const(r, width)]
        x, y, z, w = self.row(r)
        kind = x & 0xFF
        if kind == MG_SYM_CONCAT:
            return self.parts(y, w & 0xFFFF) + self.parts(z, w >> 16)
        return [self.node(r)]

    # -- nodes
    def node(self, k: int):
        if k >= self.n_nodes:
            raise ValueError(f"lane {self.i}: arena reference {k} past its {self.n_nodes} nodes")
        e = self.memo[k]
        if e is None:
            pre = self.prefix
            if pre is not None and k < len(pre):
                raw = pre[k]
                kind = self.row(k)[0] & 0xFF
                e = Bool(raw) if kind == MG_SYM_TERM and raw.width == 1 and _is_bool_op(raw) else BitVec(raw)
                self.memo[k] = e
            else:
                e = self.memo[k] = self._build(k)
        return e

    def _build(self, k: int):
        x, y, z, w = self.row(k)
        kind = x & 0xFF
        if kind == MG_SYM_BIN:
            a, c = self.ref(y), self.ref(z)
            return _mark(binary(w, a, c), kind, w, (a, c))
        if kind == MG_SYM_UN:
            a = self.ref(y)
            return _mark(unary(w, a), kind, w, (a,))
        if kind == MG_SYM_CDLOAD:
            a = self.ref(y)
            return _mark(source(kind, w, a, self.state), kind, w, (a,))
        if kind == MG_SYM_BALANCE:
            return balance_of(self.state, as_bitvec(self.ref(y)))    # no provenance, as below
        if kind == MG_SYM_ENV and (w in (MG_ENV_SELFBALANCE, MG_ENV_RETURNDATASIZE, MG_ENV_NUMBER, MG_ENV_CHAINID)
                                   or w in _FRESH):
            # no provenance: the balance and the return data change across host
            # CALLs, so a re-encoded term rides as itself, not as "the value now"
            return source(kind, w, None, self.state)
        if kind in (MG_SYM_CDSIZE, MG_SYM_ENV):
            return _mark(source(kind, w, None, self.state), kind, w, ())
        if kind == MG_SYM_CDBYTE:
            # the byte _calldata_copy_helper writes: calldata[index] (instructions.py:850-860)
            return _mark(self.state.environment.calldata[w], kind, w, (), 8)
        if kind == MG_SYM_CDBYTEX:
            # a copy from a symbolic calldata offset: calldata[simplify(offset + w)]
            # (instructions.py:816-820, 847-858)
            base = self.ref(y)
            return _mark(self.state.environment.calldata[cd_index(base, w)], kind, w, (base,), 8)
        if kind == MG_SYM_SLOAD:
            # Storage.__getitem__: simplify(Select(chain after z stores, index))
            return BitVec(_select(self.chain_raw(z), self.ref(y).raw))
        if kind == MG_SYM_EXTRACT:
            return Extract(w >> 16, w & 0xFFFF, self.node(y))
        if kind == MG_SYM_CONCAT:
            return simplify_concat(self.parts(k, x >> 8))
        if kind == MG_SYM_KECCAK:
            return keccak_of(simplify_concat(self.parts(y, w)))
        if kind == MG_SYM_TERM:
            return term(w)
        if kind == MG_SYM_MLOADK:
            # over the byte map the writes before this node made: get_word_at(offset)
            # (MLOAD), or the data SHA3 hashes, simplify(Concat(memory[offset:+w]))
            mem = self._key_memory(k)
            off = self.ref(y)
            if w == 0:
                return mem.get_word_at(off)
            data = [b if isinstance(b, BitVec) else symbol_factory.BitVecVal(b, 8)
                    for b in mem[off: off + symbol_factory.BitVecVal(w, 256)]]
            return simplify_concat(data) if len(data) > 1 else data[0]
        raise NotEncodable(f"unknown arena node kind {kind}")

    def _key_memory(self, upto: int):
        """The byte map of the MSTOREK events below node `upto`, for an MLOADK
        read: replayed incrementally (nodes decode in arena order, so each
        event is applied once per lane decode), afresh only for a read below
        the map's current point.  Reads never change the map."""
        km = getattr(self, "_kmem", None)
        if km is None or km[1] > upto:
            km = (Memory(), 0)
        mem, at = km
        for j in range(at, upto):
            # published before the event's operands decode: an MLOADK among them
            # (below j) finds the map past its point and replays afresh
            self._kmem = (mem, j)
            self._apply_key_event(mem, self.row(j))
        self._kmem = (mem, upto)
        return mem

    def _has_key_writes(self) -> bool:
        """Whether the lane's arena holds an MSTOREK event (one vectorised test
        of the node plane's kind bytes, without decoding any row)."""
        if not self.n_nodes:
            return False
        kinds = np.asarray(self.b.node[self.i, :self.n_nodes, 0]) & 0xFF
        return bool((kinds == MG_SYM_MSTOREK).any())

    def replay_keys(self, mem, upto: int) -> None:
        """Apply the lane's writes at symbolic offsets (MG_SYM_MSTOREK events of
        nodes [0, upto), in arena order = execution order) to `mem`: MSTORE's
        write_word_at, MSTORE8's low byte, a host-encoded byte (memory.py:84-115,
        instructions.py:1454-1493)."""
        for j in range(upto):
            self._apply_key_event(mem, self.row(j))

    def _apply_key_event(self, mem, row) -> None:
        x, y, z, w = row
        if x & 0xFF == MG_SYM_MSTOREK:
            off, val = self.ref(y), self.ref(z)
            if w == 1:
                mem.write_word_at(off, val)
            elif w == 2:
                mem[off] = val.value % 256 if val.value is not None else Extract(7, 0, val)
            else:
                mem[off] = val.value if val.value is not None else val

    # -- memory and storage
    def memory(self):
        """The lane's memory: concrete bytes plus the symbolic ones (memory.py
        bytes: Extract(255 - 8j, 248 - 8j, word) of a node's word)."""
        b, i = self.b, self.i
        msize = int(b.msize[i])
        symb = {}
        if hasattr(b, "mtag") and msize:
            tags = b.mtag[i, :msize]
            for p in np.flatnonzero(tags):
                t = int(tags[p]) - 1
                node, j = t >> 5, t & 31
                word = self.node(node)
                symb[int(p)] = word if word.size() == 8 else Extract(255 - 8 * j, 248 - 8 * j, word)
        mem = Memory(bytes(b.memory[i, :msize]), symb)
        if self._has_key_writes():
            self.replay_keys(mem, self.n_nodes)
        return mem

    def entry(self, e: int):
        """Storage chain entry e as (key, value).  Entries decode one at a time:
        a stored value may be a read of the chain before it (x -= v)."""
        if self._entries is None:
            self._entries = []
        b, i = self.b, self.i
        while len(self._entries) <= e:
            k = len(self._entries)
            kt, vt = (int(v) for v in b.sttag[i, k])
            key = self.node(kt - 1) if kt else symbol_factory.BitVecVal(limbs_to_word(b.storage[i, k, :8]), 256)
            val = self.node(vt - 1) if vt else symbol_factory.BitVecVal(limbs_to_word(b.storage[i, k, 8:]), 256)
            self._entries.append((key, val))
        return self._entries[e]

    def entries(self) -> list:
        """The storage chain: [(key, value)] per device entry, in store order."""
        n = int(self.b.storage_count[self.i])
        if n:
            self.entry(n - 1)
        return list(self._entries or [])[:n]

    def base_raw(self):
        acct = self.state.environment.active_account
        symstore = bool(int(self.b.flags[self.i]) & MG_LANE_SYMSTORE)
        return Storage(not symstore, acct.address).base_raw

    def chain_raw(self, m: int):
        if self._raws is None:
            self._raws = [self.base_raw()]
        while len(self._raws) <= m:
            k, v = self.entry(len(self._raws) - 1)
            self._raws.append(Node("store", 0, (self._raws[-1], k.raw, v.raw), (256, 256)))
        return self._raws[m]

    def storage(self):
        acct = self.state.environment.active_account
        symstore = bool(int(self.b.flags[self.i]) & MG_LANE_SYMSTORE)
        return Storage.from_chain(not symstore, acct.address, self.entries())


def cd_index(base, k: int) -> BitVec:
    """The calldata index _calldata_copy_helper reads byte k of a copy from a
    symbolic offset at: simplify(offset) then simplify(i + 1) per byte
    (instructions.py:816-820, 854-858) -- z3 folds the additions' constants
    into one (state.memory_key)."""
    from .state import memory_key
    raw = base.raw if k == 0 else (base + symbol_factory.BitVecVal(k, 256)).raw
    return BitVec(memory_key(raw))


def keccak_of(data):
    """KeccakFunctionManager.create_keccak's value for `data` without its
    registration: the concrete hash, or keccak256_<bits>(data)."""
    if not data.symbolic:
        from ..keccak import keccak256
        n = data.size() // 8
        return symbol_factory.BitVecVal(int.from_bytes(keccak256(data.value.to_bytes(n, "big")), "big"), 256)
    w = data.size()
    return Function(f"keccak256_{w}", [w], 256)(data)


def decode_stack(b, i: int, state, dec: Optional[_Decoder] = None) -> list:
    """Lane i's stack as the reference would hold it: BitVecVal for concrete
    words, the node's expression for symbolic ones."""
    dec = dec or _Decoder(b, i, state)
    sp = int(b.sp[i])
    tags = b.stag[i, :sp].tolist()
    raw = b.stack[i, :sp].astype("<u4", copy=False).tobytes()
    return [dec.node(t - 1) if t else symbol_factory.BitVecVal(int.from_bytes(raw[32 * s:32 * s + 32], "little"), 256)
            for s, t in enumerate(tags)]


def decode_lane(b, i: int, state, prefix: Optional[list] = None):
    """(stack, memory, storage) of a symbolic lane; `prefix`: the terms of the
    nodes its state was encoded with (LaneEncoding.enc.node_raw)."""
    dec = _Decoder(b, i, state, prefix)
    return decode_stack(b, i, state, dec), dec.memory(), dec.storage()


def decode_node(b, i: int, state, k: int):
    return _Decoder(b, i, state).node(k)


def exp_operands(b, i: int, state, k: int):
    """(base, exponent) of lane i's EXP node k (an MG_REC_SYMEXP record)."""
    dec = _Decoder(b, i, state)
    _, y, z, _ = (int(v) for v in b.node[i, k])
    return as_bitvec(dec.ref(y)), as_bitvec(dec.ref(z))


def keccak_input(b, i: int, state, k: int):
    """The input of lane i's KECCAK node k (an MG_REC_SYMKECCAK record):
    simplify(Concat(bytes)) of the hashed memory, as sha3_ passes it to
    create_keccak (instructions.py:1032-1048)."""
    dec = _Decoder(b, i, state)
    _, y, _, w = (int(v) for v in b.node[i, k])
    return simplify_concat(dec.parts(y, w))


def _concrete_value(x) -> Optional[int]:
    if isinstance(x, int):
        return x
    raw = getattr(x, "raw", None)
    if raw is not None and raw.op == "const":
        return int(raw.param)
    return None


class _Encoder:
    """One lane's arena built from expressions: nodes for expressions decode
    produced (recorded provenance) or that have the structure of a memory read,
    a keccak application or a storage read over this lane's chain; constants
    in the constant table; repeated subterms shared."""

    def __init__(self, node_cap: int = 1 << 30, const_cap: int = 1 << 30):
        self.node_cap, self.const_cap = node_cap, const_cap
        self.nodes: list = []             # (x, y, z, w)
        self.consts: list = []            # ints
        self._cref: dict = {}
        self._nref: dict = {}             # raw -> node index
        self.raws: list = []              # this lane's chain prefixes (encode_storage)
        self.node_raw: list = []          # node index -> the term it encodes

    def cref(self, v: int) -> int:
        r = self._cref.get(v)
        if r is None:
            if len(self.consts) >= self.const_cap:
                raise NotEncodable("constant table full")
            r = self._cref[v] = MG_SYM_CONST | len(self.consts)
            self.consts.append(v)
        return r

    def _push(self, raw, x, y=0, z=0, w=0) -> int:
        if len(self.nodes) >= self.node_cap:
            raise NotEncodable("arena full")
        self.nodes.append((x, y, z, w))
        self.node_raw.append(raw)
        self._nref[raw] = len(self.nodes) - 1
        return len(self.nodes) - 1

    def event(self, x, y=0, z=0, w=0) -> None:
        """An arena entry that is not a term (MG_SYM_MSTOREK)."""
        if len(self.nodes) >= self.node_cap:
            raise NotEncodable("arena full")
        self.nodes.append((x, y, z, w))
        self.node_raw.append(None)

    def enc(self, raw) -> int:
        """Operand ref of a raw term (a node index or a constant ref)."""
        if raw.op == "const":
            return self.cref(int(raw.param))
        r = self._nref.get(raw)
        if r is not None:
            return r
        prov = _PROV.get(raw)
        if prov is not None:
            kind, imm, args, width = prov
            refs = [self.enc(a.raw) for a in args]
            return self._push(raw, kind | (width << 8), refs[0] if refs else 0, refs[1] if len(refs) > 1 else 0,
                              imm)
        op = raw.op
        if op == "extract":
            src = raw.args[0]
            y = self.enc(src)
            if y & MG_SYM_CONST:
                raise NotEncodable("extract of a constant")
            hi, lo = raw.param
            return self._push(raw, MG_SYM_EXTRACT | (raw.width << 8), y, 0, (hi << 16) | lo)
        if op == "concat":
            l, r_ = raw.args
            return self._push(raw, MG_SYM_CONCAT | (raw.width << 8), self.enc(l), self.enc(r_),
                              l.width | (r_.width << 16))
        if op == "uf" and len(raw.args) == 1 and raw.param[0].startswith("keccak256_") \
                and not raw.param[0].endswith("-1") and raw.width == 256:
            return self._push(raw, MG_SYM_KECCAK | (256 << 8), self.enc(raw.args[0]), 0, raw.args[0].width)
        if op == "select" and raw.width == 256:
            arr = raw.args[0]
            for m, a in enumerate(self.raws):
                if a is arr:
                    return self._push(raw, MG_SYM_SLOAD | (256 << 8), self.enc(raw.args[1]), m, 0)
        # any other term rides on the lane as an opaque node: the device builds on
        # it and compares it by identity, the host decodes it to the same term
        if raw.width > 0xFFFFFF:
            raise NotEncodable("term too wide for an arena node")
        return self._push(raw, MG_SYM_TERM | (raw.width << 8), 0, 0, register_term(raw))

    def word(self, x) -> Tuple[int, int]:
        """(concrete value, tag) of a stack word / storage key or value."""
        v = _concrete_value(x)
        if v is not None and not isinstance(x, Bool):
            return v, 0
        if isinstance(x, Bool) and x.value is not None:
            return int(bool(x.value)), 0
        r = self.enc(x.raw)
        if r & MG_SYM_CONST:                    # a Bool folded to a constant, say
            return self.consts[r & ~MG_SYM_CONST], 0
        return 0, r + 1

    def byte(self, e) -> int:
        """Tag of a symbolic memory byte."""
        raw = e.raw
        if raw.op == "extract" and raw.width == 8 and raw.args[0].width == 256:
            hi, lo = raw.param
            if hi % 8 == 7:
                r = self.enc(raw.args[0])
                if not r & MG_SYM_CONST:
                    return 1 + ((r << 5) | ((255 - hi) // 8))
        r = self.enc(raw)
        if r & MG_SYM_CONST or raw.width != 8:
            raise NotEncodable("memory byte without arena provenance")
        return 1 + ((r << 5) | 31)


# Opaque terms of the host's expression layer carried by lanes (MG_SYM_TERM):
# index -> term, interned by identity, so equal indices are the same term.
# Lane images live only inside one LaserEVM.exec drain (states between drains
# are host objects, re-encoded when packed), so the outermost exec() clears the
# table when it starts: terms of finished transactions are not kept alive.
_TERMS: List[object] = []
_TERM_IDX: dict = {}


def reset_terms() -> None:
    _TERMS.clear()
    _TERM_IDX.clear()


def register_term(raw) -> int:
    k = _TERM_IDX.get(raw)
    if k is None:
        k = _TERM_IDX[raw] = len(_TERMS)
        _TERMS.append(raw)
    return k


def term(k: int):
    raw = _TERMS[k]
    return Bool(raw) if raw.width == 1 and raw.op not in ("const",) and _is_bool_op(raw) else BitVec(raw)


def _is_bool_op(raw) -> bool:
    return raw.op in ("eq", "distinct", "and", "or", "not", "xor", "implies", "bvult", "bvugt", "bvslt", "bvsgt",
                      "bvsle", "bvsge", "bvadd_noovfl_u", "bvumul_noovfl", "bvsub_noudfl_u") or \
        (raw.op == "var" and raw.width == 1)


class LaneEncoding:
    """Everything encode_state wrote for one state (lists, written by write())."""

    def __init__(self, enc: _Encoder, stack, mem, store, flags: int):
        self.enc, self.stack, self.mem, self.store, self.flags = enc, stack, mem, store, flags

    @property
    def symbolic(self) -> bool:
        return bool(self.flags & MG_LANE_SYMBOLIC)

    def write(self, b, i: int) -> None:
        sh = b.shape
        enc = self.enc
        if len(enc.nodes) > sh.node_cap or len(enc.consts) > sh.const_cap:
            raise NotEncodable("arena larger than the batch's capacities")
        b.stag[i] = 0
        for s, (v, t) in enumerate(self.stack):
            b.stack[i, s] = word_to_limbs(v)
            b.stag[i, s] = t
        if enc.nodes:
            b.node[i, :len(enc.nodes)] = np.array(enc.nodes, dtype=np.uint64).astype(np.uint32)
        for k, v in enumerate(enc.consts):
            b.cval[i, k] = word_to_limbs(v)
        b.n_nodes[i], b.n_consts[i] = len(enc.nodes), len(enc.consts)
        b.mtag[i] = 0
        for p, t in self.mem.items():
            b.mtag[i, p] = t
        if self.store is not None:
            if len(self.store) > sh.storage_cap:
                raise NotEncodable("storage chain longer than the batch's capacity")
            b.storage[i] = 0
            b.sttag[i] = 0
            for e, (kv, kt, vv, vt) in enumerate(self.store):
                b.storage[i, e, :8] = word_to_limbs(kv)
                b.storage[i, e, 8:] = word_to_limbs(vv)
                b.sttag[i, e] = (kt, vt)
            b.storage_count[i] = len(self.store)


def encode_state(state, node_cap: int = 1 << 30, const_cap: int = 1 << 30) -> LaneEncoding:
    """A state's stack, symbolic memory bytes and (for a symbolic lane) storage
    chain in arena form; raises NotEncodable for an expression the arena cannot
    represent.  The lane is symbolic when any of them is, or its calldata or
    environment words are, or its storage base is the symbolic Array."""
    enc = _Encoder(node_cap, const_cap)
    flags = lane_flags(state)
    storage = state.environment.active_account.storage
    symstore = not storage.concrete or (storage.is_chain and any(
        k.symbolic or v.symbolic for k, v in storage.chain()))
    store = None
    if flags or symstore or state.mstate.memory.symbolic or not all(
            _concrete_value(x) is not None or (isinstance(x, Bool) and x.value is not None)
            for x in state.mstate.stack):
        flags |= MG_LANE_SYMBOLIC
        # the chain first: storage reads on the stack refer to its prefixes
        enc.raws = [storage.base_raw]
        store = []
        for k, v in storage.chain():
            kv, kt = enc.word(k)
            vv, vt = enc.word(v)
            store.append((kv, kt, vv, vt))
            enc.raws.append(Node("store", 0, (enc.raws[-1], k.raw, v.raw), (256, 256)))
        if not storage.concrete:
            flags |= MG_LANE_SYMSTORE
        if state.environment.active_account.balance().symbolic:
            flags |= MG_LANE_SYMBAL
        env = state.environment
        if all(isinstance(w, BitVec) and w.symbolic for w in (env.block_number, env.chainid)):
            flags |= MG_LANE_SYMBLOCK
        rds = getattr(getattr(state, "last_return_data", None), "size", None)
        if isinstance(rds, BitVec) and rds.symbolic:
            flags |= MG_LANE_SYMRDS
    stack = [enc.word(x) for x in state.mstate.stack]
    mem = {}
    if state.mstate.memory.symbolic:
        for p, e in state.mstate.memory.symbolic_bytes().items():
            mem[p] = enc.byte(e)
        flags |= MG_LANE_MEMTAG
    # bytes at symbolic keys: one write event per key, in the map's order
    for key, byte in state.mstate.memory.symbolic_key_bytes().items():
        off = enc.enc(key)
        if off & MG_SYM_CONST:
            raise NotEncodable("a symbolic memory key that folds to a constant")
        val = enc.cref(byte) if isinstance(byte, int) else enc.enc(byte.raw)
        enc.event(MG_SYM_MSTOREK, off, val, 3)
    return LaneEncoding(enc, stack, mem, store, flags)


def encode_stack(b, i: int, stack: list) -> bool:
    """Write `stack` into lane i's stack rows and symbolic planes.  Returns
    whether any word is symbolic; raises NotEncodable for an expression that no
    arena node produced, or a full arena."""
    sh = b.shape
    enc = _Encoder(sh.node_cap, sh.const_cap)
    words = [enc.word(x) for x in stack]
    LaneEncoding(enc, words, {}, None, 0).write(b, i)
    return any(t for _, t in words)


def lane_flags(state) -> int:
    """MG_LANE_SYMBOLIC / MG_LANE_SYMCD / MG_LANE_SYMENV bits of a state."""
    env = state.environment
    f = 0
    if is_symbolic_calldata(env.calldata):
        f |= MG_LANE_SYMBOLIC | MG_LANE_SYMCD
    for k, attr in _ENV_ATTR.items():
        w = getattr(env, attr)
        if isinstance(w, BitVec) and w.symbolic:
            f |= MG_LANE_SYMBOLIC | (1 << (MG_LANE_SYMENV_SHIFT + k))
    return f


def state_is_symbolic(state) -> bool:
    """Whether the state needs a symbolic lane: symbolic calldata or environment
    words, a symbolic stack word or memory byte, or storage over the symbolic
    Array or with symbolic stores."""
    if lane_flags(state) or state.mstate.memory.symbolic:
        return True
    st = state.environment.active_account.storage
    if not st.concrete or (st.is_chain and any(k.symbolic or v.symbolic for k, v in st.chain())):
        return True
    return any(_concrete_value(x) is None for x in state.mstate.stack)


# ----------------------------------------------------------- JUMPI fork
def jumpi_successors(state) -> list:
    """instructions.py:1558-1636 on a state stopped at a JUMPI whose condition
    is symbolic (the target is concrete): the fall-through successor with the
    negated condition and, when the target is a JUMPDEST, the jump with the
    condition; each gets the JUMPI gas and depth + 1.  The reference also
    appends a branch condition that folds to True (every concrete JUMPI does so
    there); a lane never records those -- concrete JUMPIs run on the device --
    so a fork whose condition folded to a constant (a node the expression layer
    simplifies away) keeps that convention: True is not appended."""
    from .opcodes import get_opcode_gas
    st = state.mstate.stack
    op0, condition = st[-1], st[-2]
    jump_addr = _concrete_value(op0)
    gmin, gmax = get_opcode_gas("JUMPI")
    negated = Not(condition) if isinstance(condition, Bool) else condition == 0
    condi = condition if isinstance(condition, Bool) else condition != 0
    out = []
    if not negated.is_false:
        s = _fork_copy(state)
        _pop2(s)
        s.mstate.min_gas_used += gmin
        s.mstate.max_gas_used += gmax
        s.mstate.depth += 1
        s.mstate.pc += 1
        if negated.value is not True:       # see below: constant-true conditions are not kept
            s.world_state.constraints.append(negated)
        out.append(s)
    instrs = state.environment.code.instruction_list
    index = _instruction_index(instrs, jump_addr)
    if index is None or instrs[index]["opcode"] != "JUMPDEST":
        return out
    if not condi.is_false:
        s = _fork_copy(state)
        _pop2(s)
        s.mstate.min_gas_used += gmin
        s.mstate.max_gas_used += gmax
        s.mstate.pc = index
        s.mstate.depth += 1
        if condi.value is not True:
            s.world_state.constraints.append(condi)
        out.append(s)
    return out


def _fork_copy(state):
    """deepcopy(global_state) of the reference's fork (world state, machine
    state and account copies; expressions are immutable and shared)."""
    return copy(state)


def lane_eligible(state) -> bool:
    """Whether a lane can carry the state: every symbolic stack word, memory
    byte and storage key or value is an expression the arena represents
    (encode_state succeeds)."""
    return lane_encoding(state) is not None


def lane_encoding(state) -> Optional[LaneEncoding]:
    """encode_state(state), or None when a lane cannot carry the state (the
    batch keeps the encoding for its shape and its pack)."""
    try:
        return encode_state(state)
    except NotEncodable:
        return None


def _pop2(s):
    st = s.mstate.stack
    st.pop()
    st.pop()


_ADDRS: dict = {}        # id(instruction list) -> (the list, its addresses)


def _instruction_index(instrs, address: int) -> Optional[int]:
    """util.get_instruction_index (util.py:45-59): first index at or past address
    (a bisection over the list's addresses, which increase)."""
    got = _ADDRS.get(id(instrs))
    if got is None or got[0] is not instrs or len(got[1]) != len(instrs):
        got = _ADDRS[id(instrs)] = (instrs, [ins["address"] for ins in instrs])
    k = bisect.bisect_left(got[1], address)
    return k if k < len(instrs) else None
