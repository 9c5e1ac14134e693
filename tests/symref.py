"""CPU restatement of the reference's symbolic instruction semantics for the
paths the symbolic lanes run (test infrastructure; parity unpinned against z3:
z3 and the reference cannot be imported here).

``step(state)`` executes the instruction at ``state.mstate.pc`` the way
mythril/laser/ethereum/instructions.py does and returns the successor states,
written independently of mythril_amd/laser/symbolic.py (which turns device
arena nodes into expressions) so the two meet only in the expression layer:

* symbolic operands: the mutators of instructions.py:356-800 (pop_bitvec's
  ``If(b, 1, 0)``, Bool-valued compares, ISZERO's If, NOT as 2**256-1 - x, the
  concrete-zero divisor rules), ``get_word_at`` of SymbolicCalldata
  (state/calldata.py:214-262) and the symbolic environment words;
* a JUMPI on a symbolic condition forks as instructions.py:1558-1636 does;
* every instruction whose operands are all concrete runs on the C oracle
  (oracle/evm_ref.c, pinned on the reference's VMTests) over a concrete
  projection of the state.

* the opcodes kernel 1 leaves to the host (instructions.py:907-1000,
  1151-1440, 1700-1711, 1862-2470): BALANCE / SELFBALANCE over the world
  state's balances array, EXTCODESIZE, RETURNDATASIZE / RETURNDATACOPY,
  GAS and the block values as fresh symbols, SELFDESTRUCT, and the CALL family
  where the reference answers without running callee code -- a code-less
  callee (an ether transfer, ``transfer_ether``) or an address the disabled
  dynamic loader cannot load (``myth analyze --no-onchain-data``): symbolic
  return data and a fresh ``retval`` (call.py:36-257).  A call into code or a
  precompile raises ``Unsupported``.

An instruction with symbolic inputs outside that set raises ``Unsupported``
(a NotImplementedError, which LaserEVM drops as svm.py:314-316 does).
Halts are reported in ``Engine.ended`` as (kind, state); ``Engine.run`` is a
BFS over paths with the svm.py:319-326 fork filter, the restatement the
device-driven LaserEVM is compared against.  ``Engine(signals=True)`` is the
escape-handler form (the reference's Instruction.evaluate): halts and
exceptions are raised as TransactionEndSignal / VmException instead."""
from __future__ import annotations

from collections import Counter
from copy import copy

import numpy as np

from mythril_amd.lanes import (LaneBatch, LaneShape, MG_HALT_DROPPED, MG_HALT_END, MG_HALT_RETURN,
                               MG_HALT_REVERT, MG_HALT_STOP, MG_RUNNING, MG_VMEXC, limbs_to_word,
                               word_to_limbs)
from mythril_amd.laser.opcodes import ADDRESS_OPCODE_MAPPING
from mythril_amd.laser.state import (Account, Memory, MachineStack, OutOfGasException, VmException,
                                    WriteProtection, memory_key)
from mythril_amd.laser.transaction import ContractCreationTransaction
from mythril_amd.smt.expr import (UGE, BitVec, Bool, Concat, Extract, If, LShR, Not, SRem, UDiv, UGT, ULT,
                                  URem, simplify_concat, symbol_factory)
from mythril_amd.smt.exponent_manager import exponent_function_manager
from mythril_amd.smt.keccak_manager import keccak_function_manager
from oracle.evm_ref import OracleEVM

BVV = symbol_factory.BitVecVal


class Unsupported(NotImplementedError):
    pass


class ReturnData:
    """state/return_data.py:9-31."""

    def __init__(self, return_data, return_data_size):
        self.return_data = return_data
        self.return_data_size = return_data_size

    @property
    def size(self):
        return self.return_data_size


PRECOMPILE_COUNT = 9          # natives.py:253-265


def _z3str(x) -> str:
    """str() of a reference BitVec as the names built from it print it (z3's
    decimal for a constant)."""
    v = _val(x)
    return str(v) if v is not None else repr(getattr(x, "raw", x))


def _val(x):
    raw = getattr(x, "raw", None)
    if isinstance(x, Bool):
        return None if x.value is None else int(bool(x.value))
    return int(raw.param) if raw is not None and raw.op == "const" else None


def _pop_bitvec(x):
    """util.pop_bitvec (util.py:75-96)."""
    if isinstance(x, Bool):
        return If(x, BVV(1, 256), BVV(0, 256))
    return x


def _word_at(calldata, off):
    # BaseCalldata.get_word_at -> Concat(self[off: off + 32]); _load is
    # If(index < size (signed), calldata[index], 0)
    parts = []
    for k in range(32):
        idx = off if k == 0 else off + k
        parts.append(If(idx < calldata.size, calldata._calldata[idx], BVV(0, 8)))
    return Concat(*parts)


# pops k, pushes 1, but the pushed word is not an operation on the popped ones
# (a load from memory, storage, calldata or the environment at that index)
_NO_ANN_UNION = {"MLOAD", "SLOAD", "CALLDATALOAD", "BALANCE", "EXTCODESIZE", "EXTCODEHASH", "BLOCKHASH"}

_SYM_ENV = {0x30: "address", 0x33: "sender", 0x32: "origin", 0x34: "callvalue", 0x3A: "gasprice"}


class Engine:
    def __init__(self, pruning=None, signals: bool = False):
        self.o = OracleEVM()
        self.code_ids = {}
        self.ended = []            # (kind, state): stop / return / revert / exception / end / unsupported
        self.pruning = pruning     # callable(list of states) -> kept states (the fork filter)
        self.signals = signals     # escape-handler form: raise the reference's signals
        self.host_ops = Counter()  # opcodes stepped by the host-op restatement

    def _vmexc(self, state):
        """A VmException at `state` (the path ends without a world state)."""
        if self.signals:
            raise VmException()
        self.ended.append(("exception", state))
        return []

    # ---- concrete instructions on the oracle ---------------------------------
    def _cid(self, code):
        cid = self.code_ids.get(code.bytecode)
        if cid is None:
            raw = code.bytecode if isinstance(code.bytecode, (bytes, bytearray)) else bytes.fromhex(code.bytecode)
            cid = self.code_ids[code.bytecode] = self.o.load_code(raw)
        return cid

    def _oracle_run(self, s):
        """One instruction of the concrete projection of `s` on the oracle
        (symbolic words, memory bytes and storage read as 0 / empty): its
        status, pc, gas, depth and memory size are the instruction's whatever
        the symbolic values are (only symbolic offsets would change them, and
        those stay Unsupported)."""
        env, ms = s.environment, s.mstate
        stack = [(_val(x) or 0) for x in ms.stack]
        mem = ms.memory.raw()
        st = env.active_account.storage
        store = {} if st.is_chain else st.printable_storage
        shape = LaneShape(n=1, stack_cap=1024, mem_cap=max(4096, (len(mem) + 31) // 32 * 32 + 4096),
                          calldata_cap=32, storage_cap=max(16, 2 * len(store) + 4))
        b = LaneBatch(shape)
        b.code_id[0] = self._cid(env.code)
        b.pc[0], b.sp[0] = ms.pc, len(stack)
        for k, v in enumerate(stack):
            b.stack[0, k] = word_to_limbs(v)
        b.msize[0] = len(mem)
        b.memory[0, :len(mem)] = np.frombuffer(mem, dtype=np.uint8)
        b.depth[0] = ms.depth
        b.status[0] = MG_RUNNING
        b.gas_min[0], b.gas_max[0] = ms.min_gas_used, ms.max_gas_used
        tx = s.current_transaction
        gl = getattr(tx, "gas_limit", None)
        b.gas_limit[0] = (1 << 64) - 1 if gl is None else int(_val(gl) if not isinstance(gl, int) else gl)
        words = (env.address, env.sender, env.origin, env.callvalue, env.gasprice)
        for k, w in enumerate(words):
            b.env[0, k] = word_to_limbs(_val(w) or 0)
        for k, (key, val) in enumerate(store.items()):
            b.storage[0, k, :8] = word_to_limbs(key)
            b.storage[0, k, 8:] = word_to_limbs(val)
        b.storage_count[0] = len(store)
        self.o.run(b, max_steps=1)
        return b

    def _ended(self, s, b):
        st = int(b.status[0])
        data = bytes(b.memory[0, int(b.ret_offset[0]):int(b.ret_offset[0]) + int(b.ret_len[0])])
        if st == MG_HALT_RETURN:
            s.return_data = data
        kind = {MG_HALT_STOP: "stop", MG_HALT_RETURN: "return", MG_HALT_REVERT: "revert", MG_VMEXC: "exception",
                MG_HALT_END: "end", MG_HALT_DROPPED: "dropped"}.get(st, "unsupported")   # oracle escapes
        if self.signals:
            self._advance(s, b)
            tx = s.current_transaction
            if kind == "stop":
                tx.end(s)
            elif kind == "return":
                tx.end(s, return_data=data)
            elif kind == "revert":
                tx.end(s, return_data=data, revert=True)
            elif kind == "exception":
                raise VmException()
            elif kind == "unsupported":
                raise Unsupported("the oracle escapes this instruction")
            return []
        if kind != "dropped":
            self.ended.append((kind, s))
        return []

    def _advance(self, s, b):
        """pc, gas, depth and memory size of a completed oracle step."""
        ms = s.mstate
        ms.pc = int(b.pc[0])
        ms.depth = int(b.depth[0])
        ms.min_gas_used, ms.max_gas_used = int(b.gas_min[0]), int(b.gas_max[0])
        grow = int(b.msize[0]) - len(ms.memory)
        if grow > 0:
            ms.memory.extend(grow)

    def _oracle_step(self, s):
        env, ms = s.environment, s.mstate
        ins = env.code.instruction_list
        op_name = ins[ms.pc]["opcode"] if ms.pc < len(ins) else None
        b = self._oracle_run(s)
        if int(b.status[0]) != MG_RUNNING:
            return self._ended(s, b)
        n = s
        old = list(ms.stack)
        new_sp = int(b.sp[0])
        out = [BVV(limbs_to_word(b.stack[0, k]), 256) for k in range(new_sp)]
        # words below the instruction's reach keep their (maybe symbolic) objects
        for k in range(min(new_sp, len(old) - self._touched)):
            out[k] = old[k]
        if self._touched and new_sp == len(old) - self._touched + 1 and op_name not in _NO_ANN_UNION:
            # one word pushed for the words consumed: every BitVec operation
            # unions its operands' annotations (bitvec.py:63-136), concrete
            # operands included
            ann = frozenset().union(*(getattr(x, "annotations", frozenset()) for x in old[-self._touched:]))
            if ann:
                out[-1].annotations = out[-1].annotations | ann
        n.mstate.stack = MachineStack(out)
        # memory: the oracle's bytes; symbolic bytes stay unless the instruction
        # wrote over them (CALLDATACOPY, CODECOPY: the bytes they copied)
        sym = dict(ms.memory.symbolic_bytes())
        if sym:
            name = env.code.instruction_list[ms.pc]["opcode"]
            lo = n_w = 0
            if name in ("CALLDATACOPY", "CODECOPY"):
                lo, src, size = (_val(x) or 0 for x in (old[-1], old[-2], old[-3]))
                if name == "CALLDATACOPY":
                    n_w = size
                else:
                    code_len = len(env.code.raw)
                    n_w = min(code_len - src, size) if src < code_len else 0
            for p in range(lo, lo + n_w):
                sym.pop(p, None)
        # bytes at symbolic keys are untouched by an instruction the oracle runs
        n.mstate.memory = Memory(bytes(b.memory[0, :int(b.msize[0])]), sym, ms.memory.symbolic_key_bytes())
        n.mstate.pc = int(b.pc[0])
        n.mstate.depth = int(b.depth[0])
        n.mstate.min_gas_used, n.mstate.max_gas_used = int(b.gas_min[0]), int(b.gas_max[0])
        if op_name == "EXP":
            # exp_ appends exponent_function_manager's condition for every EXP,
            # concrete operands included (instructions.py:624-638)
            _, cond = exponent_function_manager.create_condition(_pop_bitvec(old[-1]), _pop_bitvec(old[-2]))
            n.world_state.constraints.append(cond)
        st = env.active_account.storage
        if not st.is_chain:
            st.set_slots({limbs_to_word(b.storage[0, k, :8]): limbs_to_word(b.storage[0, k, 8:])
                          for k in range(int(b.storage_count[0]))})
        return [n]

    # ---- memory, storage and SHA3 of a symbolic state ----------------------------
    def _memstore(self, s, op, state=None):
        """instructions.py:1013-1051 (sha3_), 1437-1518 (mload_ .. sstore_) on the
        host's Memory / Storage restatements (memory.py, account.py): the
        oracle's projection decides status, gas and memory size, the values are
        the reference's expressions."""
        ms, env = s.mstate, s.environment
        st = ms.stack
        if op in (0x51, 0x52, 0x53) and _val(st[-1]) is None:
            return self._symbolic_offset(state if state is not None else s, s, op)
        if op == 0x20 and _val(st[-1]) is None:
            if _val(st[-2]) is None:
                raise Unsupported("symbolic SHA3 offset and length")
            return self._symbolic_sha3(state if state is not None else s, s)
        if op == 0x20 and _val(st[-2]) is None:
            return self._symbolic_length_sha3(state if state is not None else s, s)
        b = self._oracle_run(s)
        if int(b.status[0]) != MG_RUNNING:
            return self._ended(s, b)
        self._advance(s, b)
        storage = env.active_account.storage
        if op == 0x54:
            idx = st.pop()
            st.append(storage[idx])
        elif op == 0x55:
            key, value = st.pop(), st.pop()
            storage[key] = value
        elif op == 0x51:
            off = _val(st.pop())
            st.append(ms.memory.get_word_at(off))
        elif op == 0x52:
            off, value = _val(st.pop()), st.pop()
            ms.memory.write_word_at(off, value)
        elif op == 0x53:
            off, value = _val(st.pop()), st.pop()
            v = _val(value)
            ms.memory[off] = (v % 256) if v is not None else Extract(7, 0, value)
        else:
            off, length = _val(st.pop()), _val(st.pop())
            data_list = [x if isinstance(x, BitVec) else BVV(x, 8) for x in ms.memory[off: off + length]]
            if len(data_list) > 1:
                data = simplify_concat(data_list)
            elif len(data_list) == 1:
                data = data_list[0]
            else:
                st.append(keccak_function_manager.get_empty_keccak_hash())
                return [s]
            st.append(keccak_function_manager.create_keccak(data))
        return [s]

    def _symbolic_sha3(self, state, s):
        """sha3_ (instructions.py:1014-1051) at a symbolic offset, concrete length:
        mem_extend extends nothing; the data are the bytes at the symbolic keys
        offset + k (memory.py:117-203), joined by simplify(Concat); the sha3 gas."""
        ms = s.mstate
        st = ms.stack
        index, length = st.pop(), _val(st.pop())
        if length == 0 or length > 4096:
            raise Unsupported("SHA3 length the device leaves to the host")
        g = 30 + 6 * ((length + 31) // 32)
        if ms.min_gas_used + g >= min(_gas_limit(s), 10 ** 9 + 1):
            return self._vmexc(state)
        ms.min_gas_used += g
        ms.max_gas_used += g
        data_list = [x if isinstance(x, BitVec) else BVV(x, 8) for x in ms.memory[index: index + BVV(length, 256)]]
        if len(data_list) > 1:
            data = simplify_concat(data_list)
        elif len(data_list) == 1:
            data = data_list[0]
        else:
            st.append(keccak_function_manager.get_empty_keccak_hash())
            ms.pc += 1
            return [s]
        st.append(keccak_function_manager.create_keccak(data))
        ms.pc += 1
        return [s]

    def _symbolic_length_sha3(self, state, s):
        """sha3_ (instructions.py:1014-1051) of a symbolic length at a concrete
        offset: the length is taken as 64 and `length == 64` appended to the path
        before the SHA3 gas; then mem_extend and the hash of memory[index:+64]."""
        ms = s.mstate
        st = ms.stack
        index, op1 = st.pop(), st.pop()
        if _val(index) is None or isinstance(op1, Bool):
            raise Unsupported("SHA3 of a symbolic offset and length, or of a Bool length")
        s.world_state.constraints.append(op1 == 64)
        g = 30 + 6 * 2
        if ms.min_gas_used + g >= min(_gas_limit(s), 10 ** 9 + 1):
            raise Unsupported("an out-of-gas SHA3 of a symbolic length")
        ms.min_gas_used += g
        ms.max_gas_used += g
        try:
            ms.mem_extend(index, BVV(64, 256))
        except VmException:
            return self._vmexc(state)
        data = simplify_concat([x if isinstance(x, BitVec) else BVV(x, 8)
                                for x in ms.memory[_val(index): _val(index) + 64]])
        st.append(keccak_function_manager.create_keccak(data))
        ms.pc += 1
        return [s]

    def _symbolic_offset(self, state, s, op):
        """mload_ / mstore_ / mstore8_ (instructions.py:1437-1485) at a symbolic
        offset: mem_extend extends nothing, the bytes live at symbolic keys
        (memory.py:117-203), table gas only."""
        ms = s.mstate
        st = ms.stack
        off = st.pop()
        if op == 0x51:
            st.append(ms.memory.get_word_at(off))
        elif op == 0x52:
            ms.memory.write_word_at(off, st.pop())
        else:
            v = st.pop()
            ms.memory[off] = (_val(v) % 256) if _val(v) is not None else Extract(7, 0, _pop_bitvec(v))
        gmin, gmax = _GAS[op]
        ms.min_gas_used += gmin
        ms.max_gas_used += gmax
        if ms.min_gas_used > 10 ** 9 or ms.min_gas_used >= _gas_limit(s):
            return self._vmexc(state)
        ms.pc += 1
        return [s]

    def _halt_symbolic(self, state, s, op):
        """return_ / revert_ (instructions.py:1857-1934) with a symbolic offset
        or length: the return data stays symbolic (the reference logs "not
        supported") and the transaction ends; RETURN's mem_extend of a symbolic
        range extends nothing."""
        ms = s.mstate
        off, length = ms.stack.pop(), ms.stack.pop()
        tx = s.current_transaction
        if op == 0xF3 and _val(length) is not None and ms.min_gas_used >= min(_gas_limit(s), 10 ** 9 + 1):
            return self._vmexc(state)      # mem_extend + check_gas_usage_limit (:1869-1870)
        if op == 0xF3 and isinstance(tx, ContractCreationTransaction):
            # return_ then ContractCreationTransaction.end (transaction_models.py:
            # 265-284): a symbolic length returns one fresh symbolic byte, a
            # symbolic offset the bytes at simplify(offset + k); unless every byte
            # is an int the creation installs no code (return_data None)
            n = _val(length)
            data = None
            if n is not None:
                got = ms.memory[off: off + BVV(n, 256)] if n else []
                if got and all(isinstance(x, int) for x in got):
                    data = bytes(got)
            if self.signals:
                tx.end(s, return_data=data, revert=False)
            self.ended.append(("return", s))
            return []
        if self.signals:
            tx.end(s, return_data=None, revert=op == 0xFD)
        self.ended.append(("revert" if op == 0xFD else "return", s))
        return []

    # ---- one instruction ----------------------------------------------------------
    def step(self, state):
        s = copy(state)
        ms, env = s.mstate, s.environment
        instrs = env.code.instruction_list
        if ms.pc >= len(instrs):
            self.ended.append(("end", s))
            return []
        name = instrs[ms.pc]["opcode"]
        op = next(k for k, v in ADDRESS_OPCODE_MAPPING.items() if v == name)
        st = ms.stack
        if op in _HOST_OPS:
            self.host_ops[name] += 1
            return self._host_op(state, s, op, name)
        if op in (0xF3, 0xFD) and len(st) >= 2 and (_val(st[-1]) is None or _val(st[-2]) is None):
            return self._halt_symbolic(state, s, op)
        nin = {"DUP": int(name[3:]) if name.startswith("DUP") else 0,
               "SWAP": int(name[4:]) + 1 if name.startswith("SWAP") else 0}
        reads = nin["DUP"] or nin["SWAP"] or _POPS.get(op, 0)
        sym_in = any(_val(x) is None for x in st[-reads:]) if reads and len(st) >= reads else False
        symcd = not isinstance(env.calldata, (bytes, bytearray))
        env_attr = _SYM_ENV.get(op)
        sym_env = env_attr is not None and _val(getattr(env, env_attr)) is None
        if op in (0x20, 0x51, 0x52, 0x53, 0x54, 0x55) and _symbolic_state(s) and len(st) >= _POPS[op]:
            s.environment.active_account.storage.to_chain()
            return self._memstore(s, op, state)
        creation = isinstance(s.current_transaction, ContractCreationTransaction)
        if symcd and (op == 0x37 or (creation and op in (0x38, 0x39))) and len(st) >= _POPS.get(op, 0):
            out = self._calldata_ops(state, s, op, creation)
            if out is not None:
                return out
        if name.startswith(("DUP", "SWAP")) or name == "POP" or name.startswith("PUSH"):
            self._touched = reads if not name.startswith("PUSH") else 0
            if name.startswith("DUP") or name.startswith("SWAP"):
                return self._stack_op(s, name)
            return self._oracle_step(s)
        if not (sym_in or sym_env or (symcd and op in (0x35, 0x36, 0x37))):
            self._touched = reads
            return self._oracle_step(s)
        gmin, gmax = _GAS[op]
        if op == 0x57:                                          # JUMPI
            target, cond = st[-1], st[-2]
            if _val(target) is None:
                # jumpi_ (instructions.py:1572-1579): "Skipping JUMPI to invalid
                # destination" -- both words popped, pc + 1, the JUMPI gas by hand
                st.pop(), st.pop()
                ms.pc += 1
                ms.min_gas_used += gmin
                ms.max_gas_used += gmax
                return [s]
            return self._jumpi(s, _val(target), cond)
        if op == 0x56 and _val(st[-1]) is None:
            return self._vmexc(state)     # jump_ (:1529-1532): InvalidJumpDestination
        if 0xA0 <= op <= 0xA4:
            # log_ (:1710-1723): a state mutation, then the words are popped, nothing logged
            if env.static:
                return self._vmexc(state)
            for _ in range(2 + op - 0xA0):
                st.pop()
            if ms.min_gas_used + gmin >= min(_gas_limit(s), 10 ** 9 + 1):
                return self._vmexc(state)
            ms.min_gas_used += gmin
            ms.max_gas_used += gmax
            ms.pc += 1
            return [s]
        if op == 0x37 or op not in _SYM_OK and not sym_env and op not in (0x35, 0x36, 0x0A):
            raise Unsupported(f"{name} with symbolic inputs")
        cond_after = None
        if op == 0x0A:                                          # exp_, instructions.py:624-638
            base, exponent = st.pop(), st.pop()
            if isinstance(base, Bool) or isinstance(exponent, Bool):
                raise Unsupported("EXP of a Bool")
            res, cond_after = exponent_function_manager.create_condition(base, exponent)
        elif sym_env:
            res = getattr(env, env_attr)
        elif op == 0x36:
            res = env.calldata.size
        elif op == 0x35:
            res = _word_at(env.calldata, st.pop())
        elif op == 0x15:
            v = st.pop()
            exp = Not(v) if isinstance(v, Bool) else v == 0
            res = If(exp, BVV(1, 256), BVV(0, 256))
        elif op == 0x19:
            v = st.pop()
            if isinstance(v, Bool):
                raise Unsupported("NOT of a Bool")
            res = BVV((1 << 256) - 1, 256) - v
        else:
            a, b = st.pop(), st.pop()
            res = self._binary(op, a, b)
        if len(st) + 1 > 1024:
            raise Unsupported("stack overflow")
        if ms.min_gas_used + gmin >= min(_gas_limit(s), 10 ** 9 + 1):
            return self._vmexc(state)
        if cond_after is not None:
            s.world_state.constraints.append(cond_after)
        st.append(res)
        ms.pc += 1
        ms.min_gas_used += gmin
        ms.max_gas_used += gmax
        return [s]

    # ---- opcodes kernel 1 leaves to the host --------------------------------------
    def _host_op(self, state, s, op, name):
        """StateTransition (instructions.py:98-202) around the reference's
        mutators of the opcodes kernel 1 escapes: write protection, the
        mutator, accumulate_gas with its OOG checks, pc + 1."""
        ms, env, ws = s.mstate, s.environment, s.world_state
        st = ms.stack
        gmin, gmax = _GAS[op]
        try:
            if op == 0xFF:
                if env.static:
                    raise WriteProtection()
                return self._selfdestruct(s)
            if op == 0x31:                                      # balance_ :907-931
                address = _pop_bitvec(st.pop())
                acct = ws.accounts.get(_val(address)) if _val(address) is not None else None
                if acct is not None:
                    bal = acct.balance()
                else:                     # symbolic, or the disabled loader cannot load it
                    bal = BVV(0, 256)
                    for a in ws.accounts.values():
                        bal = If(address == a.address, a.balance(), bal)
                st.append(bal)
            elif op == 0x47:                                    # selfbalance_ :968-976
                st.append(env.active_account.balance())
            elif op == 0x3B:                                    # extcodesize_ :1151-1175
                addr = st.pop()
                v = _val(addr)
                if v is None:
                    st.append(s.new_bitvec("extcodesize_" + _z3str(addr), 256))
                elif v in ws.accounts:
                    code = ws.accounts[v].code.bytecode
                    st.append(BVV(len(code) // 2 if isinstance(code, str) else len(code), 256))
                else:
                    st.append(s.new_bitvec("extcodesize_" + hex(v), 256))
            elif op == 0x3D:                                    # returndatasize_ :1359-1370
                rd = s.last_return_data
                st.append(rd.size if rd is not None else BVV(0, 256))
            elif op == 0x3E:                                    # returndatacopy_ :1314-1357
                mo, ro, size = st.pop(), st.pop(), st.pop()
                if None not in (_val(mo), _val(ro), _val(size)) and s.last_return_data is not None:
                    mo, ro, size = _val(mo), _val(ro), _val(size)
                    ms.mem_extend(BVV(mo, 256), BVV(size, 256))
                    rd = s.last_return_data
                    for i in range(size):
                        # `ro + i < rd.size`: a signed compare whose Bool is False
                        # unless it simplifies to True (bool.py:72-80)
                        inside = _val(rd.size) is not None and ro + i < _val(rd.size)
                        ms.memory[mo + i] = rd.return_data[ro + i] if inside else 0
            elif op == 0x5A:                                    # gas_ :1700-1709
                st.append(s.new_bitvec("gas", 256))
            elif op == 0x40:                                    # blockhash_ :1372-1384
                n = st.pop()
                st.append(s.new_bitvec("blockhash_block_" + _z3str(n), 256))
            elif op == 0x41:
                st.append(s.new_bitvec("coinbase", 256))
            elif op == 0x42:
                st.append(s.new_bitvec("timestamp", 256))
            elif op == 0x43:
                st.append(env.block_number)
            elif op == 0x44:
                st.append(s.new_bitvec("block_difficulty", 256))
            elif op == 0x46:
                st.append(env.chainid)
            elif op == 0x48:
                bf = env.basefee
                st.append(bf if isinstance(bf, BitVec) else BVV(int(bf or 0), 256))
            else:
                self._call(s, op)
            if len(st) > 1024:
                raise VmException()
            ms.min_gas_used += gmin
            ms.max_gas_used += gmax
            if ms.min_gas_used > 10 ** 9 or ms.min_gas_used >= _gas_limit(s):
                raise OutOfGasException()
        except VmException:
            return self._vmexc(state)
        ms.pc += 1
        return [s]

    def _call(self, s, op):
        """call_ / callcode_ / delegatecall_ / staticcall_ (instructions.py:
        1999-2470) with get_call_parameters (call.py:36-79) where no callee code
        runs: a symbolic callee or a known code-less account receives an ether
        transfer; an address the disabled dynamic loader cannot load
        (ValueError) gets nothing; both write symbolic return data and push a
        fresh retval.  A callee with code or a precompile starts a nested
        transaction / native call: Unsupported."""
        ms, env, ws = s.mstate, s.environment, s.world_state
        st = ms.stack
        with_value = op in (0xF1, 0xF2)
        instr_addr = env.code.instruction_list[ms.pc]["address"]
        gas, to = st.pop(), st.pop()
        value = st.pop() if with_value else BVV(0, 256)
        in_off, in_size, out_off, out_size = st.pop(), st.pop(), st.pop(), st.pop()
        to_v = _val(to)
        callee = None
        unloadable = False
        if to_v is None:
            callee = Account(_pop_bitvec(to), balances=ws.balances)    # get_callee_account, call.py:147-151
        elif to_v > PRECOMPILE_COUNT or to_v == 0:
            if to_v in ws.accounts:
                callee = ws.accounts[to_v]
            else:
                unloadable = True         # accounts_exist_or_load: "Dynamic Loader is deactivated"
        if not unloadable:
            code = callee.code.bytecode if callee is not None else None
            if callee is None or code not in ("", b""):
                raise Unsupported("a call into code or a precompile (a nested transaction)")
            self._transfer_ether(s, env.active_account.address, callee.address, _pop_bitvec(value))
        self._write_symbolic_returndata(s, out_off, out_size)
        st.append(s.new_bitvec("retval_" + str(instr_addr), 256))

    @staticmethod
    def _transfer_ether(s, sender, receiver, value):
        """instructions.py:74-96."""
        ws = s.world_state
        ws.constraints.append(UGE(ws.balances[sender], value))
        ws.balances[receiver] = ws.balances[receiver] + value
        ws.balances[sender] = ws.balances[sender] - value

    @staticmethod
    def _write_symbolic_returndata(s, off, size):
        """instructions.py:1961-1997."""
        if _val(off) is None or _val(size) is None:
            return
        ms = s.mstate
        off, size = _val(off), _val(size)
        data = [s.new_bitvec("call_output_var({})_{}".format((off + i) % (1 << 256), ms.pc), 8)
                for i in range(size)]
        rds = s.new_bitvec("returndatasize", 256)
        ms.mem_extend(BVV(off, 256), BVV(size, 256))
        for i in range(size):
            old = ms.memory[off + i]
            old = old if isinstance(old, BitVec) else BVV(old, 8)
            ms.memory[off + i] = If(rds >= BVV(i, 256), data[i], old)     # `i <= size`: signed
        s.last_return_data = ReturnData(data, rds)

    def _selfdestruct(self, s):
        """selfdestruct_ (instructions.py:1876-1897): the balance goes to the
        target and the transaction ends.  The reference zeroes the balance on a
        deepcopy of the account whose balance array is detached from the world
        state's (and whose balance() still reads the world state's), so the
        world state's array keeps the old balance: restated as such."""
        env, ws = s.environment, s.world_state
        target = _pop_bitvec(s.mstate.stack.pop())
        amount = env.active_account.balance()
        ws.balances[target] = ws.balances[target] + amount
        acct = copy(env.active_account)
        acct._balances = ws.balances
        acct.deleted = True
        ws._accounts[_val(acct.address)] = acct
        env.active_account = acct
        if self.signals:
            s.current_transaction.end(s)
        self.ended.append(("stop", s))
        return []

    # ---- symbolic calldata copies, a creation's calldata opcodes ---------------
    def _calldata_ops(self, state, s, op, creation):
        """calldatacopy_ / codesize_ / codecopy_ with symbolic calldata
        (instructions.py:807-891, 979-1000, 1074-1104): a creation's CALLDATACOPY
        pops three words; its CODESIZE pushes the code's size + 0x200 and pins
        calldata.size to it; a creation's CODECOPY from at or past the end of the
        code and a message call's CALLDATACOPY write calldata[src + k] into memory
        byte dst + k.  None: an ordinary code copy (the oracle runs it)."""
        ms, env = s.mstate, s.environment
        st = ms.stack
        gmin, gmax = _GAS[op]
        code_len = len(env.code.raw)
        if op == 0x38:
            n = code_len + 0x200
            if len(st) + 1 > 1024:
                raise Unsupported("stack overflow")
            s.world_state.constraints.append(env.calldata.size == BVV(n, 256))
            st.append(BVV(n, 256))
        else:
            dst, src, size = st[-1], st[-2], st[-3]
            if op == 0x39 and _val(src) is not None and _val(src) < code_len:
                return None
            skip = symsrc = False
            if op == 0x37 and not creation:
                # _calldata_copy_helper (instructions.py:807-860): a symbolic memory
                # offset copies nothing; a symbolic calldata offset reads
                # calldata[simplify(offset + k)]; a symbolic size copies
                # SYMBOLIC_CALLDATA_SIZE = 320 bytes
                if _val(dst) is None:
                    skip = True
                else:
                    symsrc = _val(src) is None
                    if _val(size) is None:
                        size = BVV(320, 256)
            if not skip and not symsrc and not (creation and op == 0x37) and \
                    any(_val(x) is None for x in (dst, src, size)):
                raise Unsupported("symbolic calldata copy operand")
            del st[-3:]
            base = src
            dst, src, size = _val(dst), _val(src), _val(size)
            if not skip and not (creation and op == 0x37) and size > 0:
                if op == 0x39:
                    src -= code_len
                if not symsrc and src + size >= 1 << 32:
                    raise Unsupported("calldata index past 2^32")
                try:
                    ms.mem_extend(BVV(dst, 256), BVV(size, 256))
                except OutOfGasException:
                    return self._vmexc(state)
                if symsrc:
                    idx = BitVec(memory_key(base.raw))            # simplify(dstart)
                    for k in range(size):
                        ms.memory[dst + k] = env.calldata[idx]
                        idx = BitVec(memory_key((idx + BVV(1, 256)).raw))     # simplify(i_data + 1)
                else:
                    for k in range(size):
                        ms.memory[dst + k] = env.calldata[src + k]
        if ms.min_gas_used + gmin >= min(_gas_limit(s), 10 ** 9 + 1):
            return self._vmexc(state)
        ms.pc += 1
        ms.min_gas_used += gmin
        ms.max_gas_used += gmax
        return [s]

    def _binary(self, op, a, b):
        if op in (0x04, 0x05, 0x06, 0x07):
            x, y = _pop_bitvec(a), _pop_bitvec(b)
            if _val(y) == 0:                                  # `if op1 == 0`: a concrete zero
                return BVV(0, 256)
            if op == 0x04:
                return UDiv(x, y)
            if op == 0x05:
                return x / y
            return URem(x, y) if op == 0x06 else SRem(x, y)
        if op == 0x01:
            return _pop_bitvec(a) + _pop_bitvec(b)
        if op == 0x02:
            return _pop_bitvec(a) * _pop_bitvec(b)
        if op == 0x03:
            return _pop_bitvec(a) - _pop_bitvec(b)
        if op == 0x10:
            return ULT(_pop_bitvec(a), _pop_bitvec(b))
        if op == 0x11:
            return UGT(_pop_bitvec(a), _pop_bitvec(b))
        if op == 0x12:
            return _pop_bitvec(a) < _pop_bitvec(b)
        if op == 0x13:
            return _pop_bitvec(a) > _pop_bitvec(b)
        if op == 0x14:
            return _pop_bitvec(a) == _pop_bitvec(b)
        if op == 0x16:
            return _pop_bitvec(a) & _pop_bitvec(b)
        if op == 0x17:
            return _pop_bitvec(a) | _pop_bitvec(b)
        if op == 0x18:
            if isinstance(a, Bool) or isinstance(b, Bool):
                raise Unsupported("XOR of a Bool")
            return a ^ b
        if op == 0x1A:
            idx = _val(a)
            if idx is None:
                raise Unsupported("symbolic BYTE index")
            off = (31 - idx) * 8
            return BVV(0, 256) if off < 0 else Concat(BVV(0, 248), Extract(off + 7, off, b))
        shift, value = _pop_bitvec(a), _pop_bitvec(b)
        if op == 0x1B:
            return value << shift
        if op == 0x1C:
            return LShR(value, shift)
        return value >> shift

    def _stack_op(self, s, name):
        st = s.mstate.stack
        k = int(name[3:]) if name.startswith("DUP") else int(name[4:])
        need = k if name.startswith("DUP") else k + 1
        if len(st) < need:
            return self._vmexc(s)
        gmin, gmax = 3, 3
        if s.mstate.min_gas_used + gmin >= min(_gas_limit(s), 10 ** 9 + 1):
            return self._vmexc(s)
        if name.startswith("DUP"):
            if len(st) + 1 > 1024:
                return self._vmexc(s)
            st.append(st[-k])
        else:
            st[-1], st[-1 - k] = st[-1 - k], st[-1]
        s.mstate.pc += 1
        s.mstate.min_gas_used += gmin
        s.mstate.max_gas_used += gmax
        return [s]

    def _jumpi(self, s, jump_addr, condition):
        """instructions.py:1558-1636."""
        gmin, gmax = 10, 10
        base = copy(s)
        base.mstate.stack.pop()
        base.mstate.stack.pop()
        negated = Not(condition) if isinstance(condition, Bool) else condition == 0
        condi = condition if isinstance(condition, Bool) else condition != 0
        out = []
        if not negated.is_false:
            n = copy(base)
            n.mstate.min_gas_used += gmin
            n.mstate.max_gas_used += gmax
            n.mstate.depth += 1
            n.mstate.pc += 1
            n.world_state.constraints.append(negated)
            out.append(n)
        instrs = s.environment.code.instruction_list
        index = next((k for k, ins in enumerate(instrs) if ins["address"] >= jump_addr), None)
        if index is None or instrs[index]["opcode"] != "JUMPDEST":
            return out
        if not condi.is_false:
            n = copy(base)
            n.mstate.min_gas_used += gmin
            n.mstate.max_gas_used += gmax
            n.mstate.pc = index
            n.mstate.depth += 1
            n.world_state.constraints.append(condi)
            out.append(n)
        return out

    # ---- BFS -----------------------------------------------------------------------
    def run(self, states, max_steps: int = 100000):
        """All paths in BFS rounds (one instruction per path per round)."""
        work = list(states)
        for _ in range(max_steps):
            if not work:
                return
            nxt = []
            for st in work:
                instrs = st.environment.code.instruction_list
                op = instrs[st.mstate.pc]["opcode"] if st.mstate.pc < len(instrs) else None
                try:
                    succ = self.step(st)
                except Unsupported as e:
                    self.ended.append(("unsupported", st))
                    continue
                if len(succ) > 1 and self.pruning is not None:
                    succ = self.pruning(succ)
                if op in ("JUMP", "JUMPI"):
                    for t in succ:
                        _switch_function(t)
                nxt.extend(succ)
            work = nxt
        raise RuntimeError("restatement did not finish")


def _switch_function(state) -> None:
    """svm.py:549-637 (manage_cfg -> _new_node_state), the function name of a
    JUMP / JUMPI successor: "constructor" in a creation, the dispatcher entry's
    name at one of its addresses, "fallback" at address 0."""
    env = state.environment
    instrs = env.code.instruction_list
    if state.mstate.pc >= len(instrs):
        return
    address = instrs[state.mstate.pc]["address"]
    seq = state.world_state.transaction_sequence
    if seq and isinstance(seq[-1], ContractCreationTransaction):
        env.active_function_name = "constructor"
    elif address in env.code.address_to_function_name:
        env.active_function_name = env.code.address_to_function_name[address]
    elif address == 0:
        env.active_function_name = "fallback"


def _symbolic_state(s) -> bool:
    """A state whose memory and storage follow the symbolic restatement (a
    symbolic lane's): symbolic calldata, environment, stack, memory or storage."""
    env = s.environment
    if not isinstance(env.calldata, (bytes, bytearray)) or s.mstate.memory.symbolic:
        return True
    if any(_val(getattr(env, a)) is None for a in _SYM_ENV.values()):
        return True
    st = env.active_account.storage
    if not st.concrete or (st.is_chain and any(_val(k) is None or _val(v) is None for k, v in st.chain())):
        return True
    return any(_val(x) is None for x in s.mstate.stack)


def _gas_limit(s):
    gl = getattr(s.current_transaction, "gas_limit", None)
    return 1 << 64 if gl is None else (gl if isinstance(gl, int) else _val(gl))


# stack words each opcode reads (the mutator's pops)
_POPS = {**{op: 2 for op in list(range(0x01, 0x08)) + [0x0A, 0x0B] + list(range(0x10, 0x15)) +
            list(range(0x16, 0x19)) + list(range(0x1A, 0x1E)) + [0x20, 0x52, 0x53, 0x55, 0x57, 0xF3, 0xFD]},
         0x08: 3, 0x09: 3, 0x15: 1, 0x19: 1, 0x35: 1, 0x37: 3, 0x39: 3, 0x3E: 3, 0x50: 1, 0x51: 1,
         0x54: 1, 0x56: 1, 0xA0: 2, 0xA1: 3, 0xA2: 4, 0xA3: 5, 0xA4: 6}
# opcodes kernel 1 escapes and the host restates (instructions.py)
_HOST_OPS = {0x31, 0x3B, 0x3D, 0x3E, 0x40, 0x41, 0x42, 0x43, 0x44, 0x46, 0x47, 0x48, 0x5A,
             0xF1, 0xF2, 0xF4, 0xFA, 0xFF}
_SYM_OK = set(range(0x01, 0x08)) | set(range(0x10, 0x15)) | {0x15, 0x16, 0x17, 0x18, 0x19, 0x1A, 0x1B, 0x1C, 0x1D}


def _gas_table():
    from mythril_amd.laser.opcodes import get_opcode_gas
    out = {}
    for op, name in ADDRESS_OPCODE_MAPPING.items():
        try:
            out[op] = tuple(get_opcode_gas(name))
        except Exception:
            out[op] = (0, 0)
    return out


_GAS = _gas_table()
