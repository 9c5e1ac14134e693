"""The seam to the reference's own objects.

Two converters a maintainer needs to put this core under an unmodified
Mythril, both duck-typed on the reference's public attributes (nothing here
imports mythril or z3):

* ``to_dag(z3_expr)`` — a z3 AST (what ``get_model`` hands quick-sat:
  ``simplify(And(*constraints)).raw``, support/model.py:52) as this repo's
  hash-consed expression DAG (mythril_amd.smt.expr), walking
  ``decl().kind()`` / ``children()`` / ``params()`` / ``sort()`` / ``as_long()``
  (the API in the reference's mypy-stubs/z3/__init__.pyi).  Operation kinds are
  looked up BY NAME (``Z3_OP_BADD`` ...) in the z3 module passed in (default:
  ``import z3``), so no numeric constant of z3 is restated here.  z3 is absent
  from this image and from the GPU box: the converter is tested on a fake AST
  (tests/fakez3.py) and is **parity unpinned** against real z3 output.
* ``pack_global_state(ref_state)`` / ``unpack_global_state`` — a reference
  ``GlobalState`` (global_state.py:21-163) whose machine state, calldata,
  environment words and active-account storage are all concrete becomes this
  repo's lane-eligible mirror GlobalState (mythril_amd.laser.state); after the
  batched engine has stepped it, the result is written back into the
  reference object.  Anything symbolic is rejected (``is_concrete`` is the
  filter): such paths stay on the reference's own ``execute_state``.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from .smt import expr as E
from .smt.expr import Node

M256 = (1 << 256) - 1


class NotConcrete(ValueError):
    """The reference state holds a symbolic value kernel 1 cannot step."""


# ======================================================================= to_dag
_BIN = {"Z3_OP_BADD": "bvadd", "Z3_OP_BSUB": "bvsub", "Z3_OP_BMUL": "bvmul",
        "Z3_OP_BUDIV": "bvudiv", "Z3_OP_BUDIV_I": "bvudiv", "Z3_OP_BUREM": "bvurem",
        "Z3_OP_BUREM_I": "bvurem", "Z3_OP_BSDIV": "bvsdiv", "Z3_OP_BSDIV_I": "bvsdiv",
        "Z3_OP_BSREM": "bvsrem", "Z3_OP_BSREM_I": "bvsrem", "Z3_OP_BSMOD": "bvsmod",
        "Z3_OP_BSMOD_I": "bvsmod", "Z3_OP_BAND": "bvand", "Z3_OP_BOR": "bvor",
        "Z3_OP_BXOR": "bvxor", "Z3_OP_BSHL": "bvshl", "Z3_OP_BLSHR": "bvlshr",
        "Z3_OP_BASHR": "bvashr"}
_NARY_BV = {"Z3_OP_BADD", "Z3_OP_BMUL", "Z3_OP_BAND", "Z3_OP_BOR", "Z3_OP_BXOR"}
_CMP = {"Z3_OP_ULT": "bvult", "Z3_OP_UGT": "bvugt", "Z3_OP_ULEQ": "bvule",
        "Z3_OP_UGEQ": "bvuge", "Z3_OP_SLT": "bvslt", "Z3_OP_SGT": "bvsgt",
        "Z3_OP_SLEQ": "bvsle", "Z3_OP_SGEQ": "bvsge"}
_UN = {"Z3_OP_BNOT": "bvnot", "Z3_OP_BNEG": "bvneg"}


class Unconvertible(ValueError):
    """A z3 operation this core does not evaluate (it stays with z3)."""


def _kinds(z3) -> Dict[int, str]:
    out = {}
    for name in dir(z3):
        if name.startswith("Z3_OP_"):
            out.setdefault(int(getattr(z3, name)), name)
    return out


def _sort_info(e, z3):
    """('bool',) | ('bv', w) | ('array', dom, rng)."""
    s = e.sort()
    k = s.kind()
    if k == z3.Z3_BOOL_SORT:
        return ("bool",)
    if k == z3.Z3_BV_SORT:
        return ("bv", s.size())
    if k == z3.Z3_ARRAY_SORT:
        return ("array", s.domain().size(), s.range().size())
    raise Unconvertible(f"sort kind {k}")


def to_dag(z3_expr, z3=None) -> Node:
    """z3 AST -> expression DAG node (Bool width 1, bit-vector width w, arrays
    as array-sorted nodes).  Shared z3 sub-terms become shared nodes."""
    if z3 is None:
        import z3  # noqa: F811  (the real module, where it is installed)
    kinds = _kinds(z3)
    memo: Dict[int, Node] = {}

    def key(e):
        return e.get_id() if hasattr(e, "get_id") else id(e)

    stack = [(z3_expr, False)]
    while stack:
        e, ready = stack.pop()
        k = key(e)
        if k in memo:
            continue
        kids = e.children()
        if not ready:
            stack.append((e, True))
            stack.extend((c, False) for c in kids if key(c) not in memo)
            continue
        memo[k] = _convert(e, [memo[key(c)] for c in kids], kinds, z3)
    return memo[key(z3_expr)]


def _convert(e, args: List[Node], kinds, z3) -> Node:
    d = e.decl()
    op = kinds.get(int(d.kind()))
    sort = _sort_info(e, z3)
    if op == "Z3_OP_BNUM":
        return E.const(int(e.as_long()), sort[1])
    if op == "Z3_OP_TRUE":
        return E.TRUE
    if op == "Z3_OP_FALSE":
        return E.FALSE
    if op == "Z3_OP_UNINTERPRETED":
        name = d.name()
        if not args:
            if sort[0] == "array":
                return Node("array", 0, (), (name, sort[1], sort[2]))
            return E.var(name, 1 if sort[0] == "bool" else sort[1])
        dom = tuple(a.width for a in args)
        return Node("uf", sort[1], tuple(args), (name, dom, sort[1]))
    if op in _BIN:
        fn = _BIN[op]
        if len(args) > 2 and op not in _NARY_BV:
            raise Unconvertible(f"{op} with {len(args)} arguments")
        acc = args[0]
        for a in args[1:]:
            acc = E._fold(fn, sort[1], (acc, a))
        return acc
    if op in _UN:
        return E._fold(_UN[op], sort[1], (args[0],))
    if op in _CMP:
        return E._fold(_CMP[op], 1, (args[0], args[1]))
    if op == "Z3_OP_EQ":
        return E._fold("eq", 1, (args[0], args[1]))
    if op == "Z3_OP_DISTINCT":
        if len(args) != 2:
            raise Unconvertible("distinct of more than two terms")
        return E._fold("distinct", 1, (args[0], args[1]))
    if op == "Z3_OP_AND":
        return E.And(*[E.Bool(a) for a in args]).raw
    if op == "Z3_OP_OR":
        return E.Or(*[E.Bool(a) for a in args]).raw
    if op == "Z3_OP_NOT":
        return E._fold("not", 1, (args[0],))
    if op == "Z3_OP_XOR":
        return E._fold("xor", 1, (args[0], args[1]))
    if op == "Z3_OP_IMPLIES":
        return E._fold("implies", 1, (args[0], args[1]))
    if op == "Z3_OP_ITE":
        if sort[0] == "bool":
            c, a, b = args
            return E.Or(E.And(E.Bool(c), E.Bool(a)), E.And(E.Not(E.Bool(c)), E.Bool(b))).raw
        if args[0] is E.TRUE:
            return args[1]
        if args[0] is E.FALSE:
            return args[2]
        return Node("ite", sort[1], tuple(args))
    if op == "Z3_OP_CONCAT":
        acc = args[0]
        for a in args[1:]:
            acc = E._fold("concat", acc.width + a.width, (acc, a))
        return acc
    if op == "Z3_OP_EXTRACT":
        hi, lo = (int(p) for p in d.params())
        return E._fold("extract", hi - lo + 1, (args[0],), (hi, lo))
    if op == "Z3_OP_ZERO_EXT":
        k = int(d.params()[0])
        return E._fold("zero_extend", args[0].width + k, (args[0],), k)
    if op == "Z3_OP_SIGN_EXT":
        k = int(d.params()[0])
        return E._fold("sign_extend", args[0].width + k, (args[0],), k)
    if op == "Z3_OP_SELECT":
        return E._select(args[0], args[1])
    if op == "Z3_OP_STORE":
        arr, i, v = args
        return Node("store", 0, (arr, i, v), (sort[1], sort[2]))
    if op == "Z3_OP_CONST_ARRAY":
        return Node("K", 0, (args[0],), (sort[1], sort[2]))
    raise Unconvertible(f"z3 operation {op or d.kind()} ({d.name()}) is not evaluated on the device")


def constraints_to_dag(z3_constraints, z3=None) -> List[E.Bool]:
    """A list of z3 Bools (e.g. [c.raw for c in constraints]) as Bool wrappers."""
    return [E.Bool(to_dag(c, z3)) for c in z3_constraints]


# ============================================================ GlobalState seam
def _val(x) -> Optional[int]:
    """int of a reference word: int, bool, or a wrapper with .value (None when
    symbolic)."""
    if isinstance(x, bool):
        return int(x)
    if isinstance(x, int):
        return x & M256
    v = getattr(x, "value", None)
    return None if v is None else int(v) & M256


def _need(x, what: str) -> int:
    v = _val(x)
    if v is None:
        raise NotConcrete(f"{what} is symbolic")
    return v


def _code_bytes(disassembly) -> bytes:
    bc = disassembly.bytecode
    if isinstance(bc, (bytes, bytearray)):
        return bytes(bc)
    bc = str(bc)
    return bytes.fromhex(bc[2:] if bc.startswith("0x") else bc)


def _calldata_bytes(cd) -> bytes:
    if isinstance(cd, (bytes, bytearray)):
        return bytes(cd)
    raw = getattr(cd, "_concrete_calldata", None)
    if raw is None:
        raise NotConcrete("calldata is symbolic (SymbolicCalldata)")
    out = bytearray()
    for k, b in enumerate(raw):
        out.append(_need(b, f"calldata byte {k}") & 0xFF)
    return bytes(out)


def _memory_bytes(mem) -> bytes:
    msize = int(getattr(mem, "_msize", len(mem)))
    buf = bytearray(msize)
    for k, v in getattr(mem, "_memory", {}).items():
        idx = _need(k, "memory index")
        if idx < msize:
            buf[idx] = _need(v, f"memory byte {idx}") & 0xFF
    return bytes(buf)


def _storage_slots(storage) -> Dict[int, int]:
    std = getattr(storage, "_standard_storage", None)
    if std is not None and type(std).__name__ != "K":
        raise NotConcrete("storage is a symbolic Array (unconstrained storage)")
    return {_need(k, "storage key"): _need(v, "storage value")
            for k, v in storage.printable_storage.items()}


def is_concrete(ref_state) -> bool:
    """True when kernel 1 can step the path: concrete stack, memory, calldata,
    environment words, transaction gas limit and K-backed active storage."""
    try:
        pack_global_state(ref_state)
        return True
    except NotConcrete:
        return False


def pack_global_state(ref_state):
    """Reference GlobalState -> this repo's mirror GlobalState (lane-eligible).
    The mirror keeps a handle on its source (``ref_state``) for write-back."""
    from .laser.disassembly import Disassembly
    from .laser.state import (Account, Environment, GlobalState, MachineState, Memory,
                              WorldState)
    from .laser.transaction import ContractCreationTransaction, MessageCallTransaction
    from .smt.expr import symbol_factory as sf

    env, ms = ref_state.environment, ref_state.mstate
    acct = env.active_account
    address = _need(acct.address, "active account address")
    code = Disassembly(_code_bytes(env.code))
    mirror_acct = Account(address, code=Disassembly(_code_bytes(acct.code)) if acct.code is not None
                          else code, contract_name=getattr(acct, "contract_name", None),
                          nonce=int(getattr(acct, "nonce", 0)))
    mirror_acct.storage.printable_storage.update(_storage_slots(acct.storage))
    bal = _val(acct.balance()) if hasattr(acct, "balance") else 0
    mirror_acct.set_balance(bal or 0)
    ws = WorldState(transaction_sequence=list(getattr(ref_state.world_state, "transaction_sequence", [])))
    ws.put_account(mirror_acct)
    calldata = _calldata_bytes(env.calldata)
    words = {name: _need(getattr(env, name), f"environment {name}")
             for name in ("sender", "origin", "callvalue", "gasprice")}
    mirror_env = Environment(mirror_acct, words["sender"], calldata, words["gasprice"],
                             words["callvalue"], words["origin"], code=code,
                             static=bool(getattr(env, "static", False)))
    stack = [sf.BitVecVal(_need(x, f"stack item {k}"), 256) for k, x in enumerate(ms.stack)]
    mstate = MachineState(gas_limit=int(ms.gas_limit), pc=int(ms.pc), stack=stack,
                          memory=Memory(_memory_bytes(ms.memory)), depth=int(ms.depth),
                          max_gas_used=int(ms.max_gas_used), min_gas_used=int(ms.min_gas_used))
    tx = ref_state.current_transaction
    gas_limit = getattr(tx, "gas_limit", None)
    gl = None if gas_limit is None else _need(gas_limit, "transaction gas limit")
    creation = type(tx).__name__ == "ContractCreationTransaction"
    cls = ContractCreationTransaction if creation else MessageCallTransaction
    mtx = cls.__new__(cls)
    MessageCallTransaction.__init__(mtx, ws, callee_account=mirror_acct, caller=words["sender"],
                                    call_data=calldata, identifier=str(getattr(tx, "id", "0")),
                                    gas_price=words["gasprice"], gas_limit=gl,
                                    origin=words["origin"], code=code, call_value=words["callvalue"],
                                    static=mirror_env.static)
    if creation:
        mtx.symbolic_calldata = False          # the packed calldata is concrete
    g = GlobalState(ws, mirror_env, None, mstate, transaction_stack=[(mtx, None)],
                    annotations=list(getattr(ref_state, "annotations", []) or []))
    g.ref_state = ref_state
    return g


def unpack_global_state(mirror, ref_state=None, symbol_factory=None):
    """Write a stepped mirror path back into its reference GlobalState: pc,
    depth, gas bounds, the stack (as the reference's BitVecVals), memory (grown
    to the mirror's size, bytes written as ints like memory.py:170-203) and the
    active account's storage (through Storage.__setitem__, so keys_set and the
    K-array stores follow).  `symbol_factory` = mythril.laser.smt.symbol_factory."""
    ref_state = ref_state if ref_state is not None else mirror.ref_state
    if symbol_factory is None:
        from mythril.laser.smt import symbol_factory  # noqa: F401  (the reference's)
    ms, rms = mirror.mstate, ref_state.mstate
    rms.pc = ms.pc
    rms.depth = ms.depth
    rms.min_gas_used, rms.max_gas_used = ms.min_gas_used, ms.max_gas_used
    del rms.stack[:]
    for w in ms.stack:
        rms.stack.append(symbol_factory.BitVecVal(_need(w, "stack"), 256))
    raw = ms.memory.raw()
    grow = len(raw) - len(rms.memory)
    if grow > 0:
        rms.memory.extend(grow)
    for k, b in enumerate(raw):
        old = rms.memory[k]
        if _val(old) != b:
            rms.memory[k] = b
    ref_storage = ref_state.environment.active_account.storage
    before = _storage_slots(ref_storage)
    for key, val in mirror.environment.active_account.storage.printable_storage.items():
        if before.get(key) != val:
            ref_storage[symbol_factory.BitVecVal(key, 256)] = symbol_factory.BitVecVal(val, 256)
    return ref_state
