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

import weakref
from copy import copy, deepcopy
from typing import List, Optional, Tuple

import numpy as np

from ..lanes import (ENV_ADDRESS as MG_ENV_ADDRESS, ENV_CALLER as MG_ENV_CALLER,
                     ENV_CALLVALUE as MG_ENV_CALLVALUE, ENV_GASPRICE as MG_ENV_GASPRICE,
                     ENV_ORIGIN as MG_ENV_ORIGIN, MG_LANE_SYMBOLIC, MG_LANE_SYMCD, MG_LANE_SYMENV_SHIFT, MG_SYM_BIN, MG_SYM_CDLOAD,
                     MG_SYM_CDSIZE, MG_SYM_CONST, MG_SYM_ENV, MG_SYM_UN, limbs_to_word, word_to_limbs)
from ..smt.expr import (Array, BitVec, Bool, Concat, Extract, If, LShR, Node, Not, UDiv, UGT, ULT, URem,
                        SRem, symbol_factory)

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

    def get_word_at(self, offset) -> BitVec:
        """BaseCalldata.get_word_at: Concat of the 32 loads at offset + k."""
        off = symbol_factory.BitVecVal(offset, 256) if isinstance(offset, int) else offset
        w = self._words.get(off.raw)
        if w is None:
            w = self._words[off.raw] = Concat(*[self._load(off if k == 0 else off + k) for k in range(32)])
        return w

    def __len__(self):
        return 0


def is_symbolic_calldata(cd) -> bool:
    return isinstance(cd, SymbolicCalldata)


# ----------------------------------------------------------- provenance
# raw node -> (kind, imm, operand expressions): what encode_stack replays
_PROV: "weakref.WeakKeyDictionary[Node, tuple]" = weakref.WeakKeyDictionary()


def _mark(e, kind: int, imm: int, args: tuple):
    """Record how node `e` was built.  A Bool result goes on the stack as
    If(b, 1, 0), as MachineStack.append wraps it (machine_state.py:39-46); the
    wrapper is what the stack holds and what encode_stack maps back to the
    (width-1) node."""
    width = 256
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
    raise NotEncodable(f"no symbolic semantics for opcode {op:#x}")


def unary(op: int, a):
    if op == 0x15:                                           # ISZERO
        exp = Not(a) if isinstance(a, Bool) else a == 0
        return If(exp, symbol_factory.BitVecVal(1, 256), symbol_factory.BitVecVal(0, 256))
    if op == 0x19:                                           # NOT: TT256M1 - x
        return symbol_factory.BitVecVal(TT256M1, 256) - a
    raise NotEncodable(f"no symbolic semantics for opcode {op:#x}")


def source(kind: int, imm: int, arg, state):
    env = state.environment
    if kind == MG_SYM_CDLOAD:
        return env.calldata.get_word_at(arg)
    if kind == MG_SYM_CDSIZE:
        return env.calldata.calldatasize
    if kind == MG_SYM_ENV:
        return getattr(env, _ENV_ATTR[imm])
    raise NotEncodable(f"unknown source kind {kind}")


# ----------------------------------------------------------- decode / encode
def decode_stack(b, i: int, state) -> list:
    """Lane i's stack as the reference would hold it: BitVecVal for concrete
    words, the node's expression for symbolic ones."""
    sp = int(b.sp[i])
    n_nodes = int(b.n_nodes[i])
    memo: List[Optional[object]] = [None] * n_nodes

    def ref(r: int):
        if r & MG_SYM_CONST:
            return symbol_factory.BitVecVal(limbs_to_word(b.cval[i, r & ~MG_SYM_CONST]), 256)
        return node(r)

    def node(k: int):
        if k >= n_nodes:
            raise ValueError(f"lane {i}: arena reference {k} past its {n_nodes} nodes")
        if memo[k] is not None:
            return memo[k]
        x, y, z, w = (int(v) for v in b.node[i, k])
        kind = x & 0xFF
        if kind == MG_SYM_BIN:
            a, c = ref(y), ref(z)
            e = _mark(binary(w, a, c), kind, w, (a, c))
        elif kind == MG_SYM_UN:
            a = ref(y)
            e = _mark(unary(w, a), kind, w, (a,))
        elif kind == MG_SYM_CDLOAD:
            a = ref(y)
            e = _mark(source(kind, w, a, state), kind, w, (a,))
        else:
            e = _mark(source(kind, w, None, state), kind, w, ())
        memo[k] = e
        return e

    out = []
    for s in range(sp):
        t = int(b.stag[i, s])
        out.append(node(t - 1) if t else symbol_factory.BitVecVal(limbs_to_word(b.stack[i, s]), 256))
    return out


def _concrete_value(x) -> Optional[int]:
    if isinstance(x, int):
        return x
    raw = getattr(x, "raw", None)
    if raw is not None and raw.op == "const":
        return int(raw.param)
    return None


def encode_stack(b, i: int, stack: list) -> bool:
    """Write `stack` into lane i's stack rows and symbolic planes.  Returns
    whether any word is symbolic; raises NotEncodable for an expression that no
    arena node produced, or a full arena."""
    sh = b.shape
    nodes: dict = {}
    consts: dict = {}
    nn = nc = 0

    def cref(v: int) -> int:
        nonlocal nc
        if v in consts:
            return consts[v]
        if nc >= sh.const_cap:
            raise NotEncodable("constant table full")
        b.cval[i, nc] = word_to_limbs(v)
        consts[v] = MG_SYM_CONST | nc
        nc += 1
        return consts[v]

    def enc(e) -> int:
        nonlocal nn
        v = _concrete_value(e)
        if v is not None and not isinstance(e, Bool):
            return cref(v)
        raw = e.raw
        if raw in nodes:
            return nodes[raw]
        prov = _PROV.get(raw)
        if prov is None:
            raise NotEncodable(f"expression without arena provenance: {raw!r}"[:200])
        kind, imm, args, width = prov
        refs = [enc(a) for a in args]
        if nn >= sh.node_cap:
            raise NotEncodable("arena full")
        b.node[i, nn] = (kind | (width << 8), refs[0] if refs else 0, refs[1] if len(refs) > 1 else 0, imm)
        nodes[raw] = nn
        nn += 1
        return nodes[raw]

    sym = False
    for s, x in enumerate(stack):
        v = _concrete_value(x)
        if v is not None and not isinstance(x, Bool):
            b.stack[i, s] = word_to_limbs(v)
            b.stag[i, s] = 0
        elif isinstance(x, Bool) and x.value is not None:
            b.stack[i, s] = word_to_limbs(int(bool(x.value)))
            b.stag[i, s] = 0
        else:
            b.stag[i, s] = enc(x) + 1
            b.stack[i, s] = 0
            sym = True
    b.n_nodes[i], b.n_consts[i] = nn, nc
    return sym


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
    if lane_flags(state):
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
    """Whether a lane can carry the state: every symbolic stack word has arena
    provenance, calldata is bytes or a SymbolicCalldata, and the active
    account's storage is concrete."""
    acct = state.environment.active_account
    if not getattr(acct.storage, "concrete", True):
        return False
    for x in state.mstate.stack:
        if _concrete_value(x) is None and not (isinstance(x, Bool) and x.value is not None):
            if x.raw not in _PROV:
                return False
    return True


def _pop2(s):
    st = s.mstate.stack
    st.pop()
    st.pop()


def _instruction_index(instrs, address: int) -> Optional[int]:
    """util.get_instruction_index (util.py:45-59): first index at or past address."""
    for k, ins in enumerate(instrs):
        if ins["address"] >= address:
            return k
    return None
