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
* ``from_dag(node, z3)`` — the other direction: a DAG node as a z3 term, built
  with z3py's own constructors (``BitVecVal``, ``UDiv``, ``Select`` ...), so
  symbolic results go back into the reference's objects.
* ``pack_global_state(ref_state, z3)`` / ``unpack_global_state`` — a reference
  ``GlobalState`` (global_state.py:21-163) becomes this repo's lane-eligible
  mirror GlobalState (mythril_amd.laser.state).  Symbolic stack words,
  environment words, memory bytes, the storage array (K or the symbolic
  ``Storage{address}`` Array with its Store chain), ``SymbolicCalldata`` and the
  path constraints are lowered with ``to_dag`` (they ride on symbolic lanes,
  laser/symbolic.py); only symbolic memory offsets and a symbolic gas limit are
  refused (``NotConcrete``: such paths stay on the reference's
  ``execute_state``).  After the batched engine has stepped the mirror, the
  result is written back into the reference object (``from_dag`` for symbolic
  values, new Stores through ``Storage.__setitem__``, new constraints appended).
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


_BOOL_OPS = {"eq", "distinct", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
             "and", "or", "not", "xor", "implies", "bvadd_noovfl_u", "bvumul_noovfl", "bvsub_noudfl_u"}


def from_dag(node: Node, z3=None, as_bool: Optional[bool] = None):
    """DAG node -> z3 term, with z3py's constructors (the module passed in;
    default ``import z3``).  Width-1 leaves are Bools where a Bool is expected
    (operands of and / or / not / ite conditions, compare results) and 1-bit
    vectors elsewhere; `as_bool` fixes the root's sort."""
    if z3 is None:
        import z3  # noqa: F811
    memo: Dict[tuple, object] = {}

    def bvsort(w):
        return z3.BitVecSort(w)

    def go(n: Node, want_bool: bool):
        key = (id(n), want_bool)
        got = memo.get(key)
        if got is not None:
            return got
        op, a = n.op, n.args
        B = lambda x: go(x, True)       # noqa: E731
        V = lambda x: go(x, False)      # noqa: E731
        if op == "const":
            out = z3.BoolVal(bool(n.param)) if (want_bool and n.width == 1) else z3.BitVecVal(n.param, n.width)
        elif op == "var":
            out = z3.Bool(n.param) if (want_bool and n.width == 1) else z3.BitVec(n.param, n.width)
        elif op == "array":
            name, dom, rng = n.param
            out = z3.Array(name, bvsort(dom), bvsort(rng))
        elif op == "K":
            out = z3.K(bvsort(n.param[0]), V(a[0]))
        elif op == "store":
            out = z3.Store(V(a[0]), V(a[1]), V(a[2]))
        elif op == "select":
            out = z3.Select(V(a[0]), V(a[1]))
        elif op == "uf":
            name, dom, rng = n.param
            out = z3.Function(name, *[bvsort(w) for w in dom], bvsort(rng))(*[V(x) for x in a])
        elif op in ("and", "or"):
            out = (z3.And if op == "and" else z3.Or)(*[B(x) for x in a])
        elif op == "not":
            out = z3.Not(B(a[0]))
        elif op == "xor":
            out = z3.Xor(B(a[0]), B(a[1]))
        elif op == "implies":
            out = z3.Implies(B(a[0]), B(a[1]))
        elif op == "ite":
            out = z3.If(B(a[0]), go(a[1], want_bool), go(a[2], want_bool))
        elif op in ("eq", "distinct"):
            bo = a[0].op in _BOOL_OPS or a[1].op in _BOOL_OPS
            x, y = go(a[0], bo), go(a[1], bo)
            out = (x == y) if op == "eq" else z3.Distinct(x, y)
        elif op == "concat":
            out = z3.Concat(V(a[0]), V(a[1]))
        elif op == "extract":
            out = z3.Extract(n.param[0], n.param[1], V(a[0]))
        elif op == "zero_extend":
            out = z3.ZeroExt(n.param, V(a[0]))
        elif op == "sign_extend":
            out = z3.SignExt(n.param, V(a[0]))
        else:
            x = V(a[0]) if a else None
            y = V(a[1]) if len(a) > 1 else None
            table = {
                "bvadd": lambda: x + y, "bvsub": lambda: x - y, "bvmul": lambda: x * y,
                "bvudiv": lambda: z3.UDiv(x, y), "bvurem": lambda: z3.URem(x, y), "bvsdiv": lambda: x / y,
                "bvsrem": lambda: z3.SRem(x, y), "bvsmod": lambda: x % y, "bvand": lambda: x & y,
                "bvor": lambda: x | y, "bvxor": lambda: x ^ y, "bvnot": lambda: ~x, "bvneg": lambda: -x,
                "bvshl": lambda: x << y, "bvlshr": lambda: z3.LShR(x, y), "bvashr": lambda: x >> y,
                "bvult": lambda: z3.ULT(x, y), "bvule": lambda: z3.ULE(x, y), "bvugt": lambda: z3.UGT(x, y),
                "bvuge": lambda: z3.UGE(x, y), "bvslt": lambda: x < y, "bvsle": lambda: x <= y,
                "bvsgt": lambda: x > y, "bvsge": lambda: x >= y,
                "bvadd_noovfl_u": lambda: z3.BVAddNoOverflow(x, y, False),
                "bvumul_noovfl": lambda: z3.BVMulNoOverflow(x, y, False),
                "bvsub_noudfl_u": lambda: z3.BVSubNoUnderflow(x, y, False),
            }
            f = table.get(op)
            if f is None:
                raise Unconvertible(f"operation {op} has no z3 constructor here")
            out = f()
        memo[key] = out
        return out

    root_bool = as_bool if as_bool is not None else node.op in _BOOL_OPS or (
        node.width == 1 and node.op in ("var", "const"))
    return go(node, root_bool)


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


def _calldata(cd):
    """bytes of a ConcreteCalldata, or this core's SymbolicCalldata for the
    reference's (the same ``{id}_calldata`` array and ``{id}_calldatasize``)."""
    if isinstance(cd, (bytes, bytearray)):
        return bytes(cd)
    raw = getattr(cd, "_concrete_calldata", None)
    if raw is None:
        from .laser.symbolic import SymbolicCalldata
        tx_id = getattr(cd, "tx_id", None)
        if tx_id is None:
            raise NotConcrete("calldata is neither concrete nor a SymbolicCalldata with a tx_id")
        return SymbolicCalldata(str(tx_id))
    out = bytearray()
    for k, b in enumerate(raw):
        out.append(_need(b, f"calldata byte {k}") & 0xFF)
    return bytes(out)


def _calldata_bytes(cd) -> bytes:
    out = _calldata(cd)
    if not isinstance(out, bytes):
        raise NotConcrete("calldata is symbolic (SymbolicCalldata)")
    return out


class _Lift:
    """Reference words -> this core's expressions: concrete values directly,
    symbolic ones through to_dag (z3 needed only then)."""

    def __init__(self, z3):
        self.z3 = z3

    def node(self, raw) -> Node:
        if self.z3 is None:
            try:
                import z3 as z  # noqa: F401  (the real module, where it is installed)
            except ImportError:
                raise NotConcrete("a symbolic value needs the z3 module to be lowered")
            self.z3 = z
        return to_dag(raw, self.z3)

    def word(self, x, what: str, width: int = 256):
        v = _val(x)
        if v is not None:
            return E.symbol_factory.BitVecVal(v, width)
        raw = getattr(x, "raw", None)
        if raw is None:
            raise NotConcrete(f"{what} is symbolic and carries no z3 term")
        n = self.node(raw)
        return E.Bool(n) if n.op in _BOOL_OPS else E.BitVec(n)


def _memory_parts(mem, lift: _Lift):
    """(concrete bytes, {offset: symbolic byte}) of a reference Memory."""
    msize = int(getattr(mem, "_msize", len(mem)))
    buf = bytearray(msize)
    sym = {}
    for k, v in getattr(mem, "_memory", {}).items():
        idx = _need(k, "memory index")
        if idx >= msize:
            continue
        b = _val(v)
        if b is None:
            sym[idx] = lift.word(v, f"memory byte {idx}", 8)
        else:
            buf[idx] = b & 0xFF
    return bytes(buf), sym


def _memory_bytes(mem) -> bytes:
    raw, sym = _memory_parts(mem, _Lift(None))
    if sym:
        raise NotConcrete("memory holds symbolic bytes")
    return raw


def _storage_slots(storage) -> Dict[int, int]:
    std = getattr(storage, "_standard_storage", None)
    if std is not None and type(std).__name__ != "K":
        raise NotConcrete("storage is a symbolic Array (unconstrained storage)")
    return {_need(k, "storage key"): _need(v, "storage value")
            for k, v in storage.printable_storage.items()}


def _storage_mirror(storage, address: int, lift: _Lift):
    """This core's Storage for a reference Storage: slot mode when it is K(0)
    plus concrete stores, else the chain of ``_standard_storage.raw`` (to_dag)
    over K(0) or the symbolic Array, store by store."""
    from .laser.state import Storage
    try:
        return Storage(True, E.symbol_factory.BitVecVal(address, 256), _storage_slots(storage))
    except NotConcrete:
        pass
    std = getattr(storage, "_standard_storage", None)
    raw = getattr(std, "raw", None)
    if raw is None:
        raise NotConcrete("symbolic storage without a z3 array term")
    n = lift.node(raw)
    entries = []
    while n.op == "store":
        entries.append((n.args[1], n.args[2]))
        n = n.args[0]
    if n.op == "K":
        if n.args[0].op != "const" or n.args[0].param != 0:
            raise NotConcrete("storage over a K array with a nonzero default")
        concrete = True
    elif n.op == "array":
        concrete = False
    else:
        raise NotConcrete(f"storage array term {n.op}")
    st = Storage.from_chain(concrete, E.symbol_factory.BitVecVal(address, 256),
                            [(E.BitVec(k), E.BitVec(v)) for k, v in reversed(entries)])
    if not concrete and n.param[0] != f"Storage{address}":
        raise NotConcrete(f"storage array named {n.param[0]}")
    return st


def is_concrete(ref_state) -> bool:
    """True when the path has no symbolic value at all (kernel 1's concrete
    lanes step it): concrete stack, memory, calldata, environment words,
    transaction gas limit and K-backed active storage."""
    try:
        _check_concrete(ref_state)
        return True
    except NotConcrete:
        return False


def _check_concrete(ref_state) -> None:
    env, ms = ref_state.environment, ref_state.mstate
    _storage_slots(env.active_account.storage)
    _calldata_bytes(env.calldata)
    for name in ("sender", "origin", "callvalue", "gasprice"):
        _need(getattr(env, name), f"environment {name}")
    for k, x in enumerate(ms.stack):
        _need(x, f"stack item {k}")
    _memory_bytes(ms.memory)
    gl = getattr(ref_state.current_transaction, "gas_limit", None)
    if gl is not None:
        _need(gl, "transaction gas limit")


def pack_global_state(ref_state, z3=None):
    """Reference GlobalState -> this repo's mirror GlobalState (lane-eligible).
    Symbolic values are lowered with to_dag (`z3`: the z3 module; default
    ``import z3``, needed only when something is symbolic).  The mirror keeps
    a handle on its source (``ref_state``) for write-back."""
    from .laser.disassembly import Disassembly
    from .laser.state import (Account, Environment, GlobalState, MachineState, Memory,
                              WorldState)
    from .laser.transaction import ContractCreationTransaction, MessageCallTransaction

    lift = _Lift(z3)
    env, ms = ref_state.environment, ref_state.mstate
    acct = env.active_account
    address = _need(acct.address, "active account address")
    code = Disassembly(_code_bytes(env.code))
    mirror_acct = Account(address, code=Disassembly(_code_bytes(acct.code)) if acct.code is not None
                          else code, contract_name=getattr(acct, "contract_name", None),
                          nonce=int(getattr(acct, "nonce", 0)))
    mirror_acct.storage = _storage_mirror(acct.storage, address, lift)
    bal = _val(acct.balance()) if hasattr(acct, "balance") else 0
    mirror_acct.set_balance(bal or 0)
    ref_cons = list(getattr(ref_state.world_state, "constraints", []) or [])
    cons = []
    for c in ref_cons:
        if isinstance(c, bool):
            cons.append(E.symbol_factory.Bool(c))
        else:
            cons.append(E.Bool(lift.node(c.raw)))
    ws = WorldState(transaction_sequence=list(getattr(ref_state.world_state, "transaction_sequence", [])),
                    constraints=cons)
    ws.put_account(mirror_acct)
    calldata = _calldata(env.calldata)
    words = {name: lift.word(getattr(env, name), f"environment {name}")
             for name in ("sender", "origin", "callvalue", "gasprice")}
    mirror_env = Environment(mirror_acct, words["sender"], calldata, words["gasprice"],
                             words["callvalue"], words["origin"], code=code,
                             static=bool(getattr(env, "static", False)))
    stack = [lift.word(x, f"stack item {k}") for k, x in enumerate(ms.stack)]
    mem, sym = _memory_parts(ms.memory, lift)
    mstate = MachineState(gas_limit=int(ms.gas_limit), pc=int(ms.pc), stack=stack,
                          memory=Memory(mem, sym), depth=int(ms.depth),
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
        mtx.symbolic_calldata = not isinstance(calldata, bytes)
    g = GlobalState(ws, mirror_env, None, mstate, transaction_stack=[(mtx, None)],
                    annotations=list(getattr(ref_state, "annotations", []) or []))
    g.ref_state = ref_state
    g.ref_n_constraints = len(ref_cons)
    g.ref_n_stores = mirror_acct.storage.n_entries() if mirror_acct.storage.is_chain else None
    return g


def unpack_global_state(mirror, ref_state=None, symbol_factory=None, smt=None, z3=None):
    """Write a stepped mirror path back into its reference GlobalState: pc,
    depth, gas bounds, the stack, memory (grown to the mirror's size; bytes as
    ints like memory.py:170-203, symbolic bytes as z3 terms), the active
    account's storage (new Stores through Storage.__setitem__, so keys_set and
    the array follow) and the path constraints added since packing.
    `symbol_factory` / `smt` = mythril.laser.smt's symbol_factory and module
    (BitVec, Bool wrap symbolic terms built by from_dag with `z3`)."""
    ref_state = ref_state if ref_state is not None else mirror.ref_state
    if symbol_factory is None:
        from mythril.laser.smt import symbol_factory  # noqa: F401  (the reference's)
    if smt is None:
        try:
            import mythril.laser.smt as smt  # noqa: F811
        except ImportError:
            smt = None

    def ref_word(w, width=256):
        v = _val(w)
        if v is not None:
            return symbol_factory.BitVecVal(v, width)
        if smt is None:
            raise NotConcrete("a symbolic value needs the reference's smt module to write back")
        return smt.BitVec(from_dag(w.raw, z3, as_bool=False))

    ms, rms = mirror.mstate, ref_state.mstate
    rms.pc = ms.pc
    rms.depth = ms.depth
    rms.min_gas_used, rms.max_gas_used = ms.min_gas_used, ms.max_gas_used
    del rms.stack[:]
    for w in ms.stack:
        rms.stack.append(ref_word(w))
    raw = ms.memory.raw()
    grow = len(raw) - len(rms.memory)
    if grow > 0:
        rms.memory.extend(grow)
    sym = ms.memory.symbolic_bytes()
    for k, b in enumerate(raw):
        if k in sym:
            rms.memory[k] = ref_word(sym[k], 8)
            continue
        old = rms.memory[k]
        if _val(old) != b:
            rms.memory[k] = b
    ref_storage = ref_state.environment.active_account.storage
    mst = mirror.environment.active_account.storage
    n0 = getattr(mirror, "ref_n_stores", None)
    if mst.is_chain and n0 is not None:
        for key, val in mst.chain()[n0:]:          # the Stores the path made, in order
            ref_storage[ref_word(key)] = ref_word(val)
    else:
        before = _storage_slots(ref_storage)
        for key, val in mst.slots().items():
            if before.get(key) != val:
                ref_storage[symbol_factory.BitVecVal(key, 256)] = symbol_factory.BitVecVal(val, 256)
    c0 = getattr(mirror, "ref_n_constraints", None)
    if c0 is not None:
        for c in mirror.world_state.constraints[c0:]:
            ref_state.world_state.constraints.append(
                smt.Bool(from_dag(c.raw, z3, as_bool=True)) if smt is not None else c)
    return ref_state
