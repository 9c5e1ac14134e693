"""Host view of a concrete LASER path: GlobalState and its parts.

Mirrors the attribute surface hooks and DetectionModules read from
mythril/laser/ethereum/state/*.py — ``state.mstate.stack[-1].value``,
``state.mstate.pc``, ``state.get_current_instruction()``,
``state.environment.active_account.storage[k]``, ``state.world_state``,
annotations — for paths whose values are all concrete.  Stack words are the
expression layer's ``BitVec`` values (mythril_amd/smt/expr.py), as LASER's are.

A GlobalState is materialised from a device lane only when the host must see
it (a hook fires, the path ends); the lane record in HBM is the state while
kernel 1 steps it.  ``to_lane``/``from_lane`` convert between the two.
"""
from __future__ import annotations

import weakref

from copy import copy
from typing import Dict, List, Optional, Union

import numpy as np

from ..smt.expr import (Array, BitVec, Bool, ConstWord, Expression, Extract, If, K, Node, _select,
                        simplify_concat, symbol_factory)
from .disassembly import Disassembly

M256 = (1 << 256) - 1
STACK_LIMIT = 1024
MSTATE_GAS_LIMIT = 1_000_000_000


# --------------------------------------------------------------- exceptions
class VmException(Exception):
    """evm_exceptions.py:4-43 (names kept so `except StackUnderflowException`
    in callers reads as in the reference)."""


class StackUnderflowException(IndexError, VmException):
    pass


class StackOverflowException(VmException):
    pass


class InvalidJumpDestination(VmException):
    pass


class InvalidInstruction(VmException):
    pass


class OutOfGasException(VmException):
    pass


class WriteProtection(VmException):
    pass


def concrete(x) -> int:
    """int of a concrete word (int, BitVec, Bool); raises for a symbolic one."""
    if isinstance(x, Expression):
        v = x.value
        if v is None:
            raise ValueError("symbolic value cannot be placed in a concrete lane")
        return int(v) & M256
    return int(x) & M256


# --------------------------------------------------------------- machine
class MachineStack(list):
    """machine_state.py:18-92: list of 256-bit words, STACK_LIMIT 1024, pop of an
    empty stack raises StackUnderflowException."""
    STACK_LIMIT = STACK_LIMIT

    def __init__(self, default_list=None):
        super().__init__(default_list or [])

    def append(self, element) -> None:
        # machine_state.py:29-56: ints become BitVecVal, Bools If(b, 1, 0)
        if isinstance(element, Bool):
            element = If(element, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
        elif not isinstance(element, BitVec):
            element = symbol_factory.BitVecVal(int(element), 256)
        if len(self) >= self.STACK_LIMIT:
            raise StackOverflowException("Reached the EVM stack limit of 1024")
        super().append(element)

    def pop(self, index=-1):
        try:
            return super().pop(index)
        except IndexError:
            raise StackUnderflowException("Trying to pop from an empty stack")

    def __getitem__(self, item):
        try:
            return super().__getitem__(item)
        except IndexError:
            raise StackUnderflowException("Trying to access a stack element which doesn't exist")

    def __add__(self, other):
        raise NotImplementedError("Implement this if needed")      # machine_state.py:80-92

    def __iadd__(self, other):
        raise NotImplementedError("Implement this if needed")


class LazyStack(MachineStack):
    """A MachineStack read back from a lane (LaserEVM._materialise): the words
    stay the lane's raw little-endian bytes until something reads an element,
    and `mut` records whether anything changed it since.  Most hook events
    never look at the stack, so they build no word objects; the raw bytes are a
    copy, so the lane's later steps cannot show through."""

    def __init__(self, raw: bytes):
        list.__init__(self)
        self._raw = raw
        self.mut = False

    def _fill(self) -> None:
        raw = self._raw
        if raw is not None:
            self._raw = None
            fb = int.from_bytes
            list.extend(self, [ConstWord(fb(raw[k: k + 32], "little")) for k in range(0, len(raw), 32)])

    def __len__(self):
        raw = self._raw
        return len(raw) >> 5 if raw is not None else list.__len__(self)

    def top_int(self, k: int) -> int:
        """int of the k-th word from the top (1 = top), without building words."""
        raw = self._raw
        if raw is not None:
            e = len(raw) - 32 * (k - 1)
            if k < 1 or e < 32:
                raise StackUnderflowException("Trying to access a stack element which doesn't exist")
            return int.from_bytes(raw[e - 32: e], "little")
        return concrete(self[-k])

    def __bool__(self):
        return len(self) > 0

    def __getitem__(self, item):
        self._fill()
        return MachineStack.__getitem__(self, item)

    def __iter__(self):
        self._fill()
        return list.__iter__(self)

    def __reversed__(self):
        self._fill()
        return list.__reversed__(self)

    def __contains__(self, x):
        self._fill()
        return list.__contains__(self, x)

    def __eq__(self, other):
        self._fill()
        return list.__eq__(self, other)

    def __ne__(self, other):
        self._fill()
        return list.__ne__(self, other)

    __hash__ = None

    def __repr__(self):
        self._fill()
        return list.__repr__(self)

    def index(self, *a):
        self._fill()
        return list.index(self, *a)

    def count(self, x):
        self._fill()
        return list.count(self, x)

    def copy(self):
        self._fill()
        return MachineStack(list.__iter__(self))

    def __copy__(self):
        return self.copy()

    def __deepcopy__(self, memo=None):
        return self.copy()

    def __reduce_ex__(self, protocol):
        return (MachineStack, (self.copy(),))

    # mutators: fill, mark, then the MachineStack / list behaviour
    def append(self, element) -> None:
        self._fill()
        self.mut = True
        MachineStack.append(self, element)

    def pop(self, index=-1):
        self._fill()
        self.mut = True
        return MachineStack.pop(self, index)

    def __setitem__(self, key, value):
        self._fill()
        self.mut = True
        list.__setitem__(self, key, value)

    def __delitem__(self, key):
        self._fill()
        self.mut = True
        list.__delitem__(self, key)

    def extend(self, it):
        self._fill()
        self.mut = True
        list.extend(self, it)

    def insert(self, i, x):
        self._fill()
        self.mut = True
        list.insert(self, i, x)

    def remove(self, x):
        self._fill()
        self.mut = True
        list.remove(self, x)

    def clear(self):
        self._fill()
        self.mut = True
        list.clear(self)

    def sort(self, *a, **k):
        self._fill()
        self.mut = True
        list.sort(self, *a, **k)

    def reverse(self):
        self._fill()
        self.mut = True
        list.reverse(self)


class Memory:
    """memory.py:28-208: a byte is an int or, for a symbolic byte, an 8-bit
    expression (``Extract(i + 7, i, value)`` of a symbolic word written with
    write_word_at, memory.py:102-115); reads of unset bytes give 0, writes at a
    concrete index >= msize are dropped (memory.py:202-203), and a word read
    with a symbolic byte in it is ``simplify(Concat(bytes))`` (memory.py:70-82,
    expr.simplify_concat).

    A symbolic index is a key of its own (the reference's dict keyed by
    ``simplify(index)``): ``memory_key`` gathers the constants of an add chain
    as z3's simplify does, so ``(p + 1) + 31`` and ``p + 32`` are one byte.
    Its ``bv_key >= len(self)`` guard is a symbolic (signed) compare that never
    drops the write.  A lane carries the bytes at symbolic keys as write events
    in its arena (MG_SYM_MSTOREK, laser/symbolic.py), replayed into this map."""

    def __init__(self, data: bytes = b"", sym: Optional[Dict[int, BitVec]] = None,
                 keys: Optional[Dict[Node, object]] = None):
        self._m = bytearray(data)
        self._sym: Dict[int, BitVec] = dict(sym) if sym else {}
        self._keys: Dict[Node, object] = dict(keys) if keys else {}     # symbolic index -> byte
        self._ver = 0            # bumped by every mutation (LaserEVM's unchanged-after-hooks test)

    def __len__(self):
        return len(self._m)

    def extend(self, size: int):
        self._ver += 1
        self._m.extend(b"\x00" * size)

    def _byte(self, k: int):
        if k >= len(self._m):
            return 0
        s = self._sym.get(k) if self._sym else None
        return self._m[k] if s is None else s

    @staticmethod
    def _index(item):
        """(int index, None) or (None, normalised symbolic key)."""
        if isinstance(item, Expression):
            if item.value is not None:
                return item.value, None
            return None, memory_key(item.raw)
        return int(item), None

    def __getitem__(self, item):
        if isinstance(item, slice):
            start, stop = item.start or 0, item.stop if item.stop is not None else len(self._m)
            if isinstance(start, Expression) or isinstance(stop, Expression):
                return [self[_add(start, k)] for k in range(_slice_len(start, stop))]
            return [self._byte(k) for k in range(start, stop)]
        k, key = self._index(item)
        if key is not None:
            return self._keys.get(key, 0)
        return self._byte(k)

    def __setitem__(self, key, value):
        k, skey = self._index(key)
        if skey is not None:
            self._ver += 1
            if isinstance(value, Expression) and value.symbolic and value.size() != 8:
                raise ValueError("a memory byte is an 8-bit expression")
            self._keys[skey] = value if isinstance(value, Expression) and value.symbolic else concrete(value) & 0xFF
            return
        if k >= len(self._m):
            return
        self._ver += 1
        if isinstance(value, Expression) and value.symbolic:
            if value.size() != 8:
                raise ValueError("a memory byte is an 8-bit expression")
            self._sym[k] = value
            self._m[k] = 0                 # the byte's concrete image (as a lane holds it)
            return
        self._m[k] = concrete(value) & 0xFF
        if self._sym:
            self._sym.pop(k, None)

    @property
    def symbolic(self) -> bool:
        return bool(self._sym) or bool(self._keys)

    @property
    def symbolic_keys(self) -> bool:
        """Bytes stored at symbolic indices (no lane can carry them)."""
        return bool(self._keys)

    def symbolic_bytes(self) -> Dict[int, BitVec]:
        """{offset: 8-bit expression} of the symbolic bytes at concrete offsets."""
        return self._sym

    def symbolic_key_bytes(self) -> Dict[Node, object]:
        """{normalised symbolic key: byte (int or 8-bit expression)}, in write order."""
        return self._keys

    def get_word_at(self, index) -> BitVec:
        k, key = self._index(index)
        if key is not None:
            parts = [self[_add(index, j)] for j in range(32)]
            if all(not isinstance(b, Expression) for b in parts):
                return symbol_factory.BitVecVal(int.from_bytes(bytes(parts), "big"), 256)
            return simplify_concat(parts)
        if self._sym and any(j in self._sym for j in range(k, k + 32)):
            return simplify_concat(self[k: k + 32])
        b = bytes(self._m[k: k + 32]).ljust(32, b"\x00") if k < len(self._m) else bytes(32)
        return symbol_factory.BitVecVal(int.from_bytes(b, "big"), 256)

    def write_word_at(self, index, value) -> None:
        k, key = self._index(index)
        pos = (lambda j: _add(index, j)) if key is not None else (lambda j: k + j)
        if isinstance(value, Expression) and value.symbolic:
            if isinstance(value, Bool):
                value = If(value, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
            for i in range(0, 256, 8):
                self[pos(31 - i // 8)] = Extract(i + 7, i, value)
            return
        v = (int(bool(value)) if isinstance(value, bool) else concrete(value)).to_bytes(32, "big")
        for j in range(32):
            self[pos(j)] = v[j]

    def raw(self) -> bytes:
        """Concrete bytes (a symbolic byte reads as 0)."""
        return bytes(self._m)

    def copy(self) -> "Memory":
        return Memory(self._m, self._sym, self._keys)

    __copy__ = copy


def memory_key(raw: Node) -> Node:
    """The key ``simplify(index)`` gives a symbolic memory index (memory.py:
    167,200): the constants of a chain of bit-vector additions summed into one
    trailing constant (0 dropped), the other operands in a canonical order (z3
    sorts the arguments of an associative-commutative operator, so ``a + b``
    and ``b + a`` are one key there too).  The order is structural (the terms'
    printed form), the same in every process, so a memory map that moved to
    another rank keys its bytes as that rank's reads do."""
    terms, c = [], 0
    stack = [raw]
    while stack:
        n = stack.pop()
        if n.op == "bvadd" and n.width == 256:
            stack.extend(reversed(n.args))
        elif n.op == "const":
            c = (c + n.param) & M256
        else:
            terms.append(n)
    if len(terms) > 1:
        terms.sort(key=_term_order)
    acc = terms[0] if terms else None
    for t in terms[1:]:
        acc = Node("bvadd", 256, (acc, t))
    if acc is None:
        return _const_node(c)
    return acc if c == 0 else Node("bvadd", 256, (acc, _const_node(c)))


_ORDER: "weakref.WeakKeyDictionary[Node, str]" = weakref.WeakKeyDictionary()


def _term_order(n: Node) -> str:
    """A structural sort key, the same on every rank: a digest computed bottom
    up over (op, width, param, child keys), memoised per node -- not repr(),
    which prints a DAG as a tree and grows ~32x per ABI nesting level of a
    calldata-derived offset."""
    k = _ORDER.get(n)
    if k is not None:
        return k
    import hashlib
    stack = [(n, False)]
    while stack:
        x, ready = stack.pop()
        if x in _ORDER:
            continue
        if not ready:
            stack.append((x, True))
            stack.extend((a, False) for a in x.args if a not in _ORDER)
            continue
        h = hashlib.blake2b(repr((x.op, x.width, x.param, tuple(_ORDER[a] for a in x.args))).encode(),
                            digest_size=12).hexdigest()
        _ORDER[x] = h
    return _ORDER[n]


def _const_node(c: int) -> Node:
    from ..smt.expr import const
    return const(c, 256)


def _add(index, j: int):
    """index + j as the reference's slice loops build it (a BitVec add)."""
    if isinstance(index, Expression):
        return index + symbol_factory.BitVecVal(j, 256) if j else index
    return index + j


def _slice_len(start, stop) -> int:
    """memory.py:137-155: the slice length when simplify(stop - start) folds to
    a constant, else APPROX_ITR + 1 = 101 entries.  Two add chains over the
    same operands differ by their constants (z3 cancels the common terms:
    (x + 40) - x is 40)."""
    d = _add(stop, 0) - start if isinstance(stop, Expression) else symbol_factory.BitVecVal(stop, 256) - start
    if d.value is not None:
        return d.value
    a, ca = _chain(stop.raw if isinstance(stop, Expression) else _const_node(stop))
    b, cb = _chain(start.raw if isinstance(start, Expression) else _const_node(start))
    if sorted(map(id, a)) == sorted(map(id, b)):
        return (ca - cb) & M256
    return 101


def _chain(raw: Node):
    """The non-constant operands and the summed constant of a bvadd chain."""
    terms, c = [], 0
    stack = [raw]
    while stack:
        n = stack.pop()
        if n.op == "bvadd" and n.width == 256:
            stack.extend(n.args)
        elif n.op == "const":
            c = (c + n.param) & M256
        else:
            terms.append(n)
    return terms, c


class MachineState:
    """machine_state.py:95-231 (concrete): pc is an instruction INDEX."""

    def __init__(self, gas_limit: int = MSTATE_GAS_LIMIT, pc: int = 0, stack=None, memory=None,
                 depth: int = 0, max_gas_used: int = 0, min_gas_used: int = 0):
        self.pc = pc
        self.stack = MachineStack(stack)
        self.memory = memory if memory is not None else Memory()
        self.gas_limit = gas_limit
        self.min_gas_used = min_gas_used
        self.max_gas_used = max_gas_used
        self.depth = depth

    @property
    def memory_size(self) -> int:
        return len(self.memory)

    def calculate_extension_size(self, start: int, size: int) -> int:
        """machine_state.py:132-146 (the old size rounds DOWN to words)."""
        if self.memory_size > start + size:
            return 0
        return ((start + size + 31) // 32 - self.memory_size // 32) * 32

    def calculate_memory_gas(self, start: int, size: int) -> int:
        """machine_state.py:148-166 (GAS_MEMORY 3, quadratic denominator 512)."""
        old = self.memory_size // 32
        new = (start + size + 31) // 32
        return (new * 3 + new * new // 512) - (old * 3 + old * old // 512)

    def check_gas(self) -> None:
        if self.min_gas_used > self.gas_limit:
            raise OutOfGasException()

    def mem_extend(self, start, size) -> None:
        """machine_state.py:171-191: a symbolic start or size extends nothing."""
        if any(isinstance(x, Expression) and x.symbolic for x in (start, size)):
            return
        start, size = concrete(start), concrete(size)
        m_extend = self.calculate_extension_size(start, size)
        if m_extend:
            gas = self.calculate_memory_gas(start, size)
            self.min_gas_used += gas
            self.max_gas_used += gas
            self.check_gas()
            self.memory.extend(m_extend)

    def pop(self, amount: int = 1):
        if amount > len(self.stack):
            raise StackUnderflowException
        values = self.stack[-amount:][::-1]
        del self.stack[-amount:]
        return values[0] if amount == 1 else values

    def __copy__(self):
        return MachineState(self.gas_limit, self.pc, list(self.stack), self.memory.copy(),
                            self.depth, self.max_gas_used, self.min_gas_used)

    __deepcopy__ = lambda self, memo=None: self.__copy__()  # noqa: E731


# --------------------------------------------------------------- accounts
class Storage:
    """account.py:18-99.  Two representations of the same array:

    * slot mode: concrete keys and values over K(256, 256, 0) as
      ``printable_storage`` {int: int} (what a concrete lane carries);
    * chain mode: the reference's ``_standard_storage`` itself -- the base array
      (K(256, 256, 0), or ``Array("Storage{address}")`` for an account without
      concrete storage) with one Store per ``__setitem__`` in order, and
      ``printable_storage`` {key: value} as expressions.  A read is
      ``simplify(Select(chain, key))`` (expr._select).  Symbolic lanes carry
      this chain (mythril_amd/laser/symbolic.py).

    A symbolic key or value, or a symbolic base, switches to chain mode; the
    slots become Stores in insertion order (the store history of keys
    overwritten while concrete is not kept: the same array, not the same
    term)."""

    def __init__(self, concrete: bool = True, address=None, slots: Optional[Dict[int, int]] = None):
        self.concrete = concrete
        self.address = address
        self.printable_storage: Dict = dict(slots or {})
        self._ver = 0                            # bumped by every mutation
        self._chain: Optional[List] = None       # [(key, value)] in store order (chain mode)
        self._raws: Optional[List] = None        # _raws[m]: the array after m stores
        if not concrete:
            self._chain, self._raws = [], [self._base_raw()]

    def _base_raw(self):
        if self.concrete:
            return K(256, 256, 0).raw
        return Array(f"Storage{concrete(self.address) if self.address is not None else None}", 256, 256).raw

    @property
    def is_chain(self) -> bool:
        return self._chain is not None

    def to_chain(self) -> "Storage":
        if self._chain is None:
            self._ver += 1
            slots = list(self.printable_storage.items())
            self._chain, self._raws, self.printable_storage = [], [self._base_raw()], {}
            for k, v in slots:
                self._append(symbol_factory.BitVecVal(k, 256), symbol_factory.BitVecVal(v, 256))
        return self

    @classmethod
    def from_chain(cls, concrete: bool, address, entries) -> "Storage":
        """Chain-mode storage with the given [(key, value)] stores in order."""
        s = cls(concrete, address)
        s._chain, s._raws, s.printable_storage = [], [s._base_raw()], {}
        for k, v in entries:
            s._append(k, v)
        return s

    def _append(self, key: BitVec, value: BitVec) -> None:
        self._ver += 1
        self._chain.append((key, value))
        self._raws.append(Node("store", 0, (self._raws[-1], key.raw, value.raw), (256, 256)))
        self.printable_storage[key] = value

    def chain(self) -> List:
        """[(key, value)] Stores in order (slot mode: its slots in insertion order)."""
        if self._chain is not None:
            return list(self._chain)
        return [(symbol_factory.BitVecVal(k, 256), symbol_factory.BitVecVal(v, 256))
                for k, v in self.printable_storage.items()]

    def chain_raw(self, m: Optional[int] = None):
        """The array term after the first m stores (all when None)."""
        self.to_chain()
        return self._raws[-1 if m is None else m]

    @property
    def base_raw(self):
        return self._raws[0] if self._raws else self._base_raw()

    def __getitem__(self, item) -> BitVec:
        if self._chain is None:
            if not (isinstance(item, Expression) and item.symbolic):
                return symbol_factory.BitVecVal(self.printable_storage.get(concrete(item), 0), 256)
            self.to_chain()
        key = item if isinstance(item, BitVec) else symbol_factory.BitVecVal(concrete(item), 256)
        return BitVec(_select(self._raws[-1], key.raw))        # array.py:21-28: no annotations

    def __setitem__(self, key, value) -> None:
        sym = any(isinstance(x, Expression) and x.symbolic for x in (key, value))
        self._ver += 1
        if self._chain is None and not sym:
            self.printable_storage[concrete(key)] = concrete(value)
            return
        self.to_chain()
        if isinstance(value, Bool):
            value = If(value, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
        k = key if isinstance(key, BitVec) else symbol_factory.BitVecVal(concrete(key), 256)
        v = value if isinstance(value, BitVec) else symbol_factory.BitVecVal(concrete(value), 256)
        self._append(k, v)

    def items(self):
        return self.printable_storage.items()

    def n_entries(self) -> int:
        return len(self._chain) if self._chain is not None else len(self.printable_storage)

    def slots(self) -> Dict[int, int]:
        """{key: value} of concrete storage (a chain of concrete stores over
        K(0), latest store per key); raises for symbolic storage."""
        if self._chain is None:
            return self.printable_storage
        if not self.concrete:
            raise ValueError("symbolic storage cannot be placed in a concrete lane")
        out: Dict[int, int] = {}
        for k, v in self._chain:
            out[concrete(k)] = concrete(v)
        return out

    def set_slots(self, slots: Dict[int, int]) -> None:
        """Replace the contents by concrete slots (slot mode)."""
        self._ver += 1
        self._chain = self._raws = None
        self.__dict__.pop("_pending", None)
        self.printable_storage = dict(slots)

    def set_slots_raw(self, raw: bytes) -> None:
        """set_slots from a lane's storage rows (64 bytes per slot: key then value,
        little-endian limbs); the dict is built on first use of printable_storage."""
        self._ver += 1
        self._chain = self._raws = None
        self.__dict__.pop("printable_storage", None)
        self._pending = raw

    def __getattr__(self, name):
        if name == "printable_storage":
            raw = self.__dict__.pop("_pending", None)
            if raw is not None:
                fb = int.from_bytes
                d = self.printable_storage = {fb(raw[k: k + 32], "little"): fb(raw[k + 32: k + 64], "little")
                                              for k in range(0, len(raw), 64)}
                return d
        raise AttributeError(name)

    def __copy__(self):
        s = Storage(self.concrete, self.address, None)
        s.printable_storage = dict(self.printable_storage)
        if self._chain is not None:
            s._chain, s._raws = list(self._chain), list(self._raws)
        else:
            s._chain = s._raws = None
        return s


class Account:
    """account.py:102-228.  The balance is ``balances[address]`` over the world
    state's symbolic ``Array("balance")`` (world_state.py:31-33), as in the
    reference: concrete balances are stores into it, so a path's balance
    arithmetic and the ``UGE(balances[sender], value)`` conjunct of every
    transaction are the reference's terms.  An account not yet put into a world
    state keeps a balance set on it and hands it over on put_account."""

    def __init__(self, address, code: Optional[Disassembly] = None, contract_name: str = None,
                 balances=None, concrete_storage: bool = True, dynamic_loader=None, nonce: int = 0):
        self.address = symbol_factory.BitVecVal(concrete(address), 256) if not isinstance(
            address, BitVec) else address
        self.nonce = nonce
        self.code = code or Disassembly("")
        if contract_name is None:
            # account.py:139-146
            contract_name = ("{0:#0{1}x}".format(self.address.value, 42) if self.address.value is not None
                             else "unknown")
        self.contract_name = contract_name
        self.concrete_storage = concrete_storage
        self.storage = Storage(concrete_storage, address=self.address)
        self.deleted = False
        self._balances = balances
        self._pending_balance = None

    def balance(self) -> BitVec:
        if self._balances is None:
            return symbol_factory.BitVecVal(concrete(self._pending_balance or 0), 256)
        return self._balances[self.address]

    def set_balance(self, balance) -> None:
        balance = balance if isinstance(balance, BitVec) else symbol_factory.BitVecVal(concrete(balance), 256)
        if self._balances is None:
            self._pending_balance = balance
            return
        self._balances[self.address] = balance

    def add_balance(self, balance) -> None:
        balance = balance if isinstance(balance, BitVec) else symbol_factory.BitVecVal(concrete(balance), 256)
        if self._balances is None:
            self._pending_balance = (self._pending_balance or symbol_factory.BitVecVal(0, 256)) + balance
            return
        self._balances[self.address] = self._balances[self.address] + balance

    def __copy__(self):
        a = Account(self.address, self.code, self.contract_name, balances=copy(self._balances),
                    concrete_storage=self.concrete_storage, nonce=self.nonce)
        a.storage = copy(self.storage)
        a.deleted = self.deleted
        a._pending_balance = self._pending_balance
        return a


class WorldState:
    """world_state.py:18-242: accounts, the symbolic ``balances`` array and its
    ``starting_balances`` copy, path constraints, transaction sequence,
    annotations."""

    def __init__(self, transaction_sequence=None, annotations=None, constraints=None):
        self._accounts: Dict[int, Account] = {}
        self.balances = Array("balance", 256, 256)
        self.starting_balances = copy(self.balances)
        self.constraints = list(constraints or [])
        self.transaction_sequence = list(transaction_sequence or [])
        self._annotations = list(annotations or [])
        self.node = None

    @property
    def accounts(self) -> Dict[int, Account]:
        return self._accounts

    def put_account(self, account: Account) -> None:
        """world_state.py:249-255 (an account's balance lives in this world
        state's array from now on)."""
        self._accounts[concrete(account.address)] = account
        pending = account._pending_balance if account._balances is None else None
        account._balances = self.balances
        account._pending_balance = None
        if pending is not None:
            account.set_balance(pending)

    def __getitem__(self, item) -> Account:
        """world_state.py:43-57: an unknown address gets a fresh account."""
        key = concrete(item)
        try:
            return self._accounts[key]
        except KeyError:
            acct = Account(item if isinstance(item, BitVec) else key, balances=self.balances)
            self._accounts[key] = acct
            return acct

    def __copy__(self):
        # __init__'s fields without its fresh balance arrays (replaced right away)
        w = WorldState.__new__(WorldState)
        w._accounts = {}
        w.constraints = list(self.constraints)
        w.transaction_sequence = list(self.transaction_sequence)
        w._annotations = [copy(a) for a in self._annotations]
        w.balances = copy(self.balances)
        w.starting_balances = copy(self.starting_balances)
        for k, a in self._accounts.items():
            c = copy(a)
            c._balances = w.balances
            w._accounts[k] = c
        w.node = self.node
        return w

    @property
    def annotations(self):
        return self._annotations

    def annotate(self, annotation) -> None:
        self._annotations.append(annotation)

    def get_annotations(self, annotation_type: type):
        return filter(lambda x: isinstance(x, annotation_type), self._annotations)


class Environment:
    """environment.py:12-60 (concrete words)."""

    def __init__(self, active_account: Account, sender, calldata: bytes, gasprice, callvalue, origin,
                 basefee=0, code: Optional[Disassembly] = None, static: bool = False):
        self.active_account = active_account
        self.active_function_name = ""
        self.address = active_account.address
        self.code = active_account.code if code is None else code
        self.sender = sender if isinstance(sender, BitVec) else symbol_factory.BitVecVal(concrete(sender), 256)
        # bytes (ConcreteCalldata) or a laser.symbolic.SymbolicCalldata
        self.calldata = calldata if hasattr(calldata, "get_word_at") else bytes(calldata)
        self.gasprice = gasprice if isinstance(gasprice, BitVec) else symbol_factory.BitVecVal(
            concrete(gasprice), 256)
        self.callvalue = callvalue if isinstance(callvalue, BitVec) else symbol_factory.BitVecVal(
            concrete(callvalue), 256)
        self.origin = origin if isinstance(origin, BitVec) else symbol_factory.BitVecVal(concrete(origin), 256)
        self.basefee = basefee
        self.static = static
        # environment.py:47-48: always symbolic
        self.block_number = symbol_factory.BitVecSym("block_number", 256)
        self.chainid = symbol_factory.BitVecSym("chain_id", 256)

    def __copy__(self):
        # every field as it is (the words are immutable expressions; __init__
        # would only rebuild the same block_number / chain_id symbols)
        e = Environment.__new__(Environment)
        e.__dict__.update(self.__dict__)
        return e


# --------------------------------------------------------------- global state
class GlobalState:
    """global_state.py:18-163: one path.  ``lane`` is the host-side handle of the
    device lane this state is mirrored into during LaserEVM.exec."""

    def __init__(self, world_state: WorldState, environment: Environment, node=None,
                 machine_state: Optional[MachineState] = None, transaction_stack=None,
                 last_return_data=None, annotations=None):
        self.node = node
        self.world_state = world_state
        self.environment = environment
        self.mstate = machine_state if machine_state else MachineState(gas_limit=MSTATE_GAS_LIMIT)
        self.transaction_stack = transaction_stack if transaction_stack else []
        self.op_code = ""
        self.last_return_data = last_return_data
        self._annotations = annotations or []
        self.lane_steps = 0          # instructions executed on the device in this exec()

    def add_annotations(self, annotations: List) -> None:
        self._annotations += annotations

    def new_bitvec(self, name: str, size: int = 256, annotations=None) -> BitVec:
        """global_state.py:146-156: a fresh symbol named after the current
        transaction."""
        return symbol_factory.BitVecSym("{}_{}".format(self.current_transaction.id, name), size,
                                        annotations=annotations)

    def __copy__(self) -> "GlobalState":
        world_state = copy(self.world_state)
        environment = copy(self.environment)
        environment.active_account = world_state[concrete(environment.active_account.address)]
        g = GlobalState(world_state, environment, self.node, copy(self.mstate),
                        transaction_stack=copy(self.transaction_stack),
                        last_return_data=self.last_return_data,
                        annotations=[copy(a) for a in self._annotations])
        g.lane_steps = self.lane_steps
        return g

    @property
    def accounts(self) -> Dict:
        return self.world_state._accounts

    def get_current_instruction(self) -> Dict:
        return self.environment.code.instruction_list[self.mstate.pc]

    @property
    def instruction(self) -> Dict:
        return self.get_current_instruction()

    @property
    def current_transaction(self):
        try:
            return self.transaction_stack[-1][0]
        except IndexError:
            return None

    @property
    def annotations(self) -> List:
        return self._annotations

    def annotate(self, annotation) -> None:
        self._annotations.append(annotation)
        if getattr(annotation, "persist_to_world_state", False):
            self.world_state.annotate(annotation)

    def get_annotations(self, annotation_type: type):
        return filter(lambda x: isinstance(x, annotation_type), self.annotations)


Word = Union[int, BitVec]
