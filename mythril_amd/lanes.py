"""Host image of a batch of concrete EVM lanes (the mg_lane_soa of include/mythgpu.h).

One lane is one LASER path in the concrete subset: the fields mirror what the
reference keeps in a GlobalState (state/global_state.py:21-56):
MachineState pc/stack/memory/gas/depth (state/machine_state.py:95-231), the active
account's concrete storage (state/account.py:18-99), ConcreteCalldata
(state/calldata.py:121-165) and the Environment words (state/environment.py:12-60).

Layout is lane-major numpy arrays; ``LaneBatch.soa()`` wraps them in the ctypes
struct the C-ABI takes.  256-bit words are 8 little-endian uint32 limbs.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Sequence

import numpy as np

# ---- constants mirrored from include/mythgpu.h -------------------------------
MG_RUNNING, MG_HALT_STOP, MG_HALT_RETURN, MG_HALT_REVERT = 0, 1, 2, 3
MG_HALT_END, MG_HALT_DROPPED, MG_VMEXC, MG_HOOK, MG_ESCAPE, MG_DEPTH = 4, 5, 6, 7, 8, 9
MG_LOOP_BOUND = 10
MG_FORK = 11            # JUMPI on a symbolic condition (symbolic lanes)
STATUS_NAMES = {
    MG_RUNNING: "running", MG_HALT_STOP: "stop", MG_HALT_RETURN: "return",
    MG_HALT_REVERT: "revert", MG_HALT_END: "end", MG_HALT_DROPPED: "dropped",
    MG_VMEXC: "vmexception", MG_HOOK: "hook", MG_ESCAPE: "escape", MG_DEPTH: "depth",
    MG_LOOP_BOUND: "loop_bound",
}
# statuses after which the reference keeps the world state (svm.py:384-389, 452-460)
WORLD_STATE_KEPT = (MG_HALT_STOP, MG_HALT_RETURN, MG_HALT_END)

MG_EXC_STACK_UNDERFLOW, MG_EXC_STACK_OVERFLOW, MG_EXC_INVALID_JUMP = 1, 2, 3
MG_EXC_INVALID_INSTRUCTION, MG_EXC_OUT_OF_GAS, MG_EXC_WRITE_PROTECTION = 4, 5, 6
MG_ESC_OPCODE, MG_ESC_MEMORY, MG_ESC_STORAGE, MG_ESC_STACK, MG_ESC_TRACE = 1, 2, 3, 4, 5
MG_ESC_RECORD = 6
MG_ESC_SYMBOLIC, MG_ESC_ARENA, MG_ESC_TAINT = 7, 8, 9
MG_RET_SYMBOLIC = 0xFFFFFFFF
MG_FENT_NONE = 0xFFFFFFFF   # no JUMP / JUMPI landed on a function entry since the upload
# function-manager records (include/mythgpu.h MG_REC_*)
MG_REC_KECCAK, MG_REC_EXP, MG_REC_ANNOT, MG_REC_HOOK, MG_REC_HEADER = 1, 2, 3, 4, 11
MG_REC_SYMKECCAK = 5    # SHA3 of a symbolic input: payload = the KECCAK node's index
MG_REC_CDSIZE = 6       # a creation's CODESIZE: the host appends calldata.size == result
MG_REC_SYMEXP = 7       # EXP with a symbolic operand: payload = the Power node's index
MG_REC_SYMLEN = 8       # SHA3 of a symbolic length: payload = the length's node; host appends len == 64
MG_REC_ANNOT_WORDS = MG_REC_HEADER + 11

MG_LANE_STATIC, MG_LANE_CREATION, MG_LANE_HOOK_ACK, MG_LANE_STEP1 = 1, 2, 4, 8
MG_LANE_SYMBOLIC, MG_LANE_SYMCD, MG_LANE_SYMENV_SHIFT = 16, 32, 6
MG_SYM_CDLOAD, MG_SYM_CDSIZE, MG_SYM_ENV, MG_SYM_BIN, MG_SYM_UN = 1, 2, 3, 4, 5
MG_SYM_SLOAD, MG_SYM_KECCAK, MG_SYM_EXTRACT, MG_SYM_CONCAT, MG_SYM_TERM = 6, 7, 8, 9, 10
MG_SYM_CDBYTE = 12      # calldata[w]: one byte of a symbolic calldata copy
MG_SYM_CDBYTEX = 13     # calldata[simplify(y + w)]: a copy from a symbolic calldata offset
MG_SYM_MSTOREK = 14     # event: write of value ref z at symbolic offset y (w: 1 word, 2 low byte, 3 byte)
MG_SYM_MLOADK = 15      # get_word_at(y) over the byte map of the events before it
MG_SYM_BALANCE = 16     # balance_ of the address ref y over the world state's accounts
MG_LANE_SYMSTORE, MG_LANE_MEMTAG = 4096, 8192
MG_LANE_SYMBAL, MG_LANE_SYMRDS, MG_LANE_BALANCE = 32768, 65536, 131072
MG_ENV_SELFBALANCE, MG_ENV_RETURNDATASIZE, MG_ENV_GAS = 5, 6, 7
MG_ENV_COINBASE, MG_ENV_TIMESTAMP, MG_ENV_DIFFICULTY, MG_ENV_NUMBER, MG_ENV_CHAINID = 8, 9, 10, 11, 12
MG_LANE_SYMBLOCK = 262144
MG_LANE_RETDATA = 16384
MG_SYM_CONST = 0x80000000
MG_LANE_TAINT = 2048
# taint action word (include/mythgpu.h MG_TAINT_*)
MG_TAINT_POST, MG_TAINT_EXPCOND, MG_TAINT_YCLASS = 16, 32, 64
MG_TAINT_SINK_SHIFT, MG_TAINT_YIELD_SHIFT = 8, 12
MG_TAINT_DEFER_SHIFT, MG_TAINT_IFSYM_SHIFT, MG_TAINT_IFLANE = 16, 20, 1 << 24
MG_TAINT_OBJ0 = 7
MG_TAINT_CDSIZE = 6     # handle of the symbolic calldata-size object
ENV_ADDRESS, ENV_CALLER, ENV_ORIGIN, ENV_CALLVALUE, ENV_GASPRICE = range(5)
MG_ENV_WORDS = 5
MG_STACK_LIMIT = 1024
MSTATE_GAS_LIMIT = 1_000_000_000

M256 = (1 << 256) - 1


def word_to_limbs(x: int) -> np.ndarray:
    return np.frombuffer((int(x) & M256).to_bytes(32, "little"), dtype="<u4").astype(np.uint32)


def limbs_to_word(l: Sequence[int]) -> int:
    if isinstance(l, np.ndarray) and l.dtype == np.uint32 and l.size == 8:
        return int.from_bytes(l.astype("<u4", copy=False).tobytes(), "little")
    return sum(int(v) << (32 * k) for k, v in enumerate(l))


def rows_to_words(rows: np.ndarray) -> list:
    """(n, 8) uint32 limbs -> n ints (one bytes conversion for the block)."""
    raw = np.ascontiguousarray(rows, dtype="<u4").tobytes()
    return [int.from_bytes(raw[32 * k: 32 * k + 32], "little") for k in range(rows.shape[0])]


def words_to_limbs(xs: Iterable[int]) -> np.ndarray:
    """Vectorised int -> (n, 8) uint32."""
    xs = list(xs)
    out = np.zeros((len(xs), 8), dtype=np.uint32)
    for i, x in enumerate(xs):
        x &= M256
        b = x.to_bytes(32, "little")
        out[i] = np.frombuffer(b, dtype="<u4")
    return out


class MgLaneSoa(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32), ("stack_cap", ctypes.c_uint32), ("mem_cap", ctypes.c_uint32),
        ("calldata_cap", ctypes.c_uint32), ("storage_cap", ctypes.c_uint32),
        ("_pad", ctypes.c_uint32),
        ("code_id", ctypes.c_void_p), ("pc", ctypes.c_void_p), ("sp", ctypes.c_void_p),
        ("msize", ctypes.c_void_p), ("depth", ctypes.c_void_p), ("status", ctypes.c_void_p),
        ("aux", ctypes.c_void_p), ("steps", ctypes.c_void_p), ("flags", ctypes.c_void_p),
        ("gas_min", ctypes.c_void_p), ("gas_max", ctypes.c_void_p), ("gas_limit", ctypes.c_void_p),
        ("calldata_len", ctypes.c_void_p), ("calldata", ctypes.c_void_p), ("env", ctypes.c_void_p),
        ("stack", ctypes.c_void_p), ("memory", ctypes.c_void_p),
        ("storage_count", ctypes.c_void_p), ("storage", ctypes.c_void_p),
        ("ret_offset", ctypes.c_void_p), ("ret_len", ctypes.c_void_p),
        ("trace_cap", ctypes.c_uint32), ("_pad2", ctypes.c_uint32),
        ("trace_len", ctypes.c_void_p), ("trace", ctypes.c_void_p),
        ("rec_cap", ctypes.c_uint32), ("_pad3", ctypes.c_uint32),
        ("rec_len", ctypes.c_void_p), ("rec", ctypes.c_void_p),
        ("fent", ctypes.c_void_p),
    ]


class MgSymSoa(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("stack_cap", ctypes.c_uint32), ("node_cap", ctypes.c_uint32),
                ("const_cap", ctypes.c_uint32), ("stag", ctypes.c_void_p), ("node", ctypes.c_void_p),
                ("cval", ctypes.c_void_p), ("n_nodes", ctypes.c_void_p), ("n_consts", ctypes.c_void_p),
                ("mem_cap", ctypes.c_uint32), ("storage_cap", ctypes.c_uint32),
                ("mtag", ctypes.c_void_p), ("sttag", ctypes.c_void_p)]


_SYM_FIELDS = ("stag", "node", "cval", "n_nodes", "n_consts", "mtag", "sttag")


class MgTaintSoa(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("stack_cap", ctypes.c_uint32), ("obj_cap", ctypes.c_uint32),
                ("_pad", ctypes.c_uint32), ("sobj", ctypes.c_void_p), ("omask", ctypes.c_void_p),
                ("n_obj", ctypes.c_void_p), ("n_fixed", ctypes.c_void_p), ("n_atoms", ctypes.c_void_p),
                ("sink", ctypes.c_void_p), ("ymask", ctypes.c_void_p), ("tflags", ctypes.c_void_p)]


_TAINT_FIELDS = ("sobj", "omask", "n_obj", "n_fixed", "n_atoms", "sink", "ymask", "tflags")

_U32_FIELDS = ("code_id", "pc", "sp", "msize", "depth", "status", "aux", "steps", "flags",
               "calldata_len", "storage_count", "ret_offset", "ret_len", "trace_len", "rec_len", "fent")
_U64_FIELDS = ("gas_min", "gas_max", "gas_limit")


@dataclass
class LaneShape:
    n: int
    stack_cap: int = MG_STACK_LIMIT
    mem_cap: int = 1024
    calldata_cap: int = 128
    storage_cap: int = 16
    trace_cap: int = 0
    rec_cap: int = 0
    node_cap: int = 0        # symbolic lanes: arena nodes per lane (0: no symbolic planes)
    const_cap: int = 0       # symbolic lanes: constant-table entries per lane
    obj_cap: int = 0         # taint lanes: object handles per lane (0: no taint planes)

    def __post_init__(self):
        if self.mem_cap % 32:
            raise ValueError("mem_cap must be a multiple of 32")
        if not 0 < self.stack_cap <= MG_STACK_LIMIT:
            raise ValueError("stack_cap must be in 1..1024")


class LaneBatch:
    """Lane-major numpy image of ``n`` lanes."""

    def __init__(self, shape: LaneShape):
        self.shape = shape
        n = shape.n
        for f in _U32_FIELDS:
            setattr(self, f, np.zeros(n, dtype=np.uint32))
        for f in _U64_FIELDS:
            setattr(self, f, np.zeros(n, dtype=np.uint64))
        self.fent[:] = MG_FENT_NONE
        self.calldata = np.zeros((n, shape.calldata_cap), dtype=np.uint8)
        self.env = np.zeros((n, MG_ENV_WORDS, 8), dtype=np.uint32)
        self.stack = np.zeros((n, shape.stack_cap, 8), dtype=np.uint32)
        self.memory = np.zeros((n, shape.mem_cap), dtype=np.uint8)
        self.storage = np.zeros((n, shape.storage_cap, 16), dtype=np.uint32)
        self.trace = np.zeros((n, max(shape.trace_cap, 1)), dtype=np.uint32)
        self.rec = np.zeros((n, max(shape.rec_cap, 1)), dtype=np.uint32)
        if shape.node_cap:
            self.stag = np.zeros((n, shape.stack_cap), dtype=np.uint32)
            self.node = np.zeros((n, shape.node_cap, 4), dtype=np.uint32)
            self.cval = np.zeros((n, max(shape.const_cap, 1), 8), dtype=np.uint32)
            self.n_nodes = np.zeros(n, dtype=np.uint32)
            self.n_consts = np.zeros(n, dtype=np.uint32)
            # byte tags of memory (0 = concrete, else 1 + (node << 5 | j): byte j of
            # the node's word) and (key, value) tags of the storage chain entries
            self.mtag = np.zeros((n, shape.mem_cap), dtype=np.uint32)
            self.sttag = np.zeros((n, shape.storage_cap, 2), dtype=np.uint32)
        if shape.obj_cap:
            self.sobj = np.zeros((n, shape.stack_cap), dtype=np.uint32)
            self.omask = np.zeros((n, shape.obj_cap), dtype=np.uint64)
            self.n_obj = np.full(n, MG_TAINT_OBJ0, dtype=np.uint32)
            self.n_fixed = np.full(n, MG_TAINT_OBJ0, dtype=np.uint32)
            self.n_atoms = np.zeros(n, dtype=np.uint32)
            self.sink = np.zeros(n, dtype=np.uint64)
            self.ymask = np.zeros(n, dtype=np.uint64)
            self.tflags = np.zeros(n, dtype=np.uint32)

    @property
    def symbolic(self) -> bool:
        return self.shape.node_cap > 0

    @property
    def taint(self) -> bool:
        return self.shape.obj_cap > 0

    def taint_soa_range(self, first: int, n: int) -> MgTaintSoa:
        """mg_taint_soa over lanes [first, first + n) (taint planes)."""
        if first < 0 or n < 0 or first + n > self.shape.n:
            raise ValueError("lane range out of bounds")
        s = MgTaintSoa()
        s.n, s.stack_cap, s.obj_cap = n, self.shape.stack_cap, self.shape.obj_cap
        for f in _TAINT_FIELDS:
            arr = getattr(self, f)
            setattr(s, f, arr.ctypes.data + first * arr.strides[0])
        self._keep_taint = s
        return s

    def sym_soa_range(self, first: int, n: int) -> MgSymSoa:
        """mg_sym_soa over lanes [first, first + n) (symbolic planes)."""
        if first < 0 or n < 0 or first + n > self.shape.n:
            raise ValueError("lane range out of bounds")
        s = MgSymSoa()
        s.n, s.stack_cap = n, self.shape.stack_cap
        s.node_cap, s.const_cap = self.shape.node_cap, self.shape.const_cap
        s.mem_cap, s.storage_cap = self.shape.mem_cap, self.shape.storage_cap
        for f in _SYM_FIELDS:
            arr = getattr(self, f)
            setattr(s, f, arr.ctypes.data + first * arr.strides[0])
        self._keep_sym = s
        return s

    @property
    def n(self) -> int:
        return self.shape.n

    # ---- ctypes view ---------------------------------------------------
    def soa(self) -> MgLaneSoa:
        s = MgLaneSoa()
        s.n = self.shape.n
        s.stack_cap, s.mem_cap = self.shape.stack_cap, self.shape.mem_cap
        s.calldata_cap, s.storage_cap = self.shape.calldata_cap, self.shape.storage_cap
        s.trace_cap = self.shape.trace_cap
        s.rec_cap = self.shape.rec_cap
        for f in _U32_FIELDS + _U64_FIELDS + ("calldata", "env", "stack", "memory", "storage",
                                              "trace", "rec"):
            arr = getattr(self, f)
            assert arr.flags["C_CONTIGUOUS"]
            setattr(s, f, arr.ctypes.data)
        self._keep = s  # keep the struct alive with the arrays
        return s

    def soa_range(self, first: int, n: int) -> MgLaneSoa:
        """Struct over lanes [first, first + n) of this image (for partial
        mg_lanes_upload / mg_lanes_download of the lanes the host touched)."""
        if first < 0 or n < 0 or first + n > self.shape.n:
            raise ValueError("lane range out of bounds")
        s = MgLaneSoa()
        s.n = n
        s.stack_cap, s.mem_cap = self.shape.stack_cap, self.shape.mem_cap
        s.calldata_cap, s.storage_cap = self.shape.calldata_cap, self.shape.storage_cap
        s.trace_cap = self.shape.trace_cap
        s.rec_cap = self.shape.rec_cap
        for f in _U32_FIELDS + _U64_FIELDS + ("calldata", "env", "stack", "memory", "storage",
                                              "trace", "rec"):
            arr = getattr(self, f)
            setattr(s, f, arr.ctypes.data + first * arr.strides[0])
        self._keep_range = s
        return s

    def copy(self) -> "LaneBatch":
        out = LaneBatch(self.shape)
        for f in _U32_FIELDS + _U64_FIELDS + ("calldata", "env", "stack", "memory", "storage",
                                              "trace", "rec") + (_SYM_FIELDS if self.symbolic else ()) + (
                                                  _TAINT_FIELDS if self.taint else ()):
            getattr(out, f)[...] = getattr(self, f)
        return out

    def regrown(self, shape: "LaneShape") -> "LaneBatch":
        """The same lanes in a batch of larger capacities (same n, calldata_cap,
        and symbolic / taint planes): every per-lane table is copied as a prefix
        (stack, memory, storage, trace, records, arena and object tables are
        filled from index 0 up), so the lanes continue where they stopped."""
        if shape.n != self.shape.n or shape.calldata_cap != self.shape.calldata_cap or \
                bool(shape.node_cap) != self.symbolic or bool(shape.obj_cap) != self.taint:
            raise ValueError("regrown: only capacities may change")
        out = LaneBatch(shape)
        for f in _U32_FIELDS + _U64_FIELDS + ("calldata", "env", "stack", "memory", "storage", "trace",
                                              "rec") + (_SYM_FIELDS if self.symbolic else ()) + (
                                                  _TAINT_FIELDS if self.taint else ()):
            src, dst = getattr(self, f), getattr(out, f)
            if src.ndim == 1:
                dst[...] = src
            else:
                k = min(src.shape[1], dst.shape[1])
                if k < src.shape[1]:
                    raise ValueError(f"regrown: {f} would shrink")
                dst[:, :k] = src[:, :k]
        return out

    # ---- per-lane construction ----------------------------------------
    def set_lane(self, i: int, *, code_id: int = 0, calldata: bytes = b"",
                 address: int = 0, caller: int = 0, origin: int = 0, callvalue: int = 0,
                 gasprice: int = 0, gas_limit: int = 8_000_000,
                 storage: Optional[Dict[int, int]] = None, flags: int = 0) -> None:
        """Initial state of a concrete message call, as transaction/concolic.py:75-122
        builds it: pc 0, empty stack and memory, gas 0, depth 0."""
        if len(calldata) > self.shape.calldata_cap:
            raise ValueError("calldata longer than calldata_cap")
        storage = storage or {}
        if len(storage) > self.shape.storage_cap:
            raise ValueError("more initial storage slots than storage_cap")
        self.code_id[i] = code_id
        self.pc[i] = self.sp[i] = self.msize[i] = self.depth[i] = 0
        self.status[i] = MG_RUNNING
        self.aux[i] = self.steps[i] = 0
        self.fent[i] = MG_FENT_NONE
        self.flags[i] = flags
        self.gas_min[i] = self.gas_max[i] = 0
        self.gas_limit[i] = gas_limit
        self.calldata[i] = 0
        self.calldata[i, : len(calldata)] = np.frombuffer(bytes(calldata), dtype=np.uint8)
        self.calldata_len[i] = len(calldata)
        for k, v in ((ENV_ADDRESS, address), (ENV_CALLER, caller), (ENV_ORIGIN, origin),
                     (ENV_CALLVALUE, callvalue), (ENV_GASPRICE, gasprice)):
            self.env[i, k] = word_to_limbs(v)
        self.storage[i] = 0
        for s, (k, v) in enumerate(storage.items()):
            self.storage[i, s, :8] = word_to_limbs(k)
            self.storage[i, s, 8:] = word_to_limbs(v)
        self.storage_count[i] = len(storage)
        self.stack[i] = 0
        self.memory[i] = 0
        self.ret_offset[i] = self.ret_len[i] = 0

    # ---- per-lane inspection ------------------------------------------
    def stack_words(self, i: int):
        return [limbs_to_word(self.stack[i, k]) for k in range(int(self.sp[i]))]

    def storage_dict(self, i: int, drop_zero: bool = True) -> Dict[int, int]:
        out = {}
        for s in range(int(self.storage_count[i])):
            k = limbs_to_word(self.storage[i, s, :8])
            v = limbs_to_word(self.storage[i, s, 8:])
            out[k] = v
        if drop_zero:
            out = {k: v for k, v in out.items() if v}
        return out

    def records(self, i: int, start: int = 0):
        """Lane i's function-manager records in execution order, as (step, kind, ...):
        (step, "keccak", input bytes, hash) and (step, "exp", base, exponent, result),
        step = the lane's steps count before the instruction."""
        out = []
        q = self.rec[i, : int(self.rec_len[i])]
        k = start
        while k < q.size:
            kind, ln, step = int(q[k]), int(q[k + 1]), int(q[k + 2])
            r = limbs_to_word(q[k + 3: k + 11])
            k += MG_REC_HEADER
            if kind == MG_REC_KECCAK:
                nw = (ln + 3) // 4
                data = q[k: k + nw].astype(">u4").tobytes()[:ln]
                out.append((step, "keccak", data, r))
                k += nw
            elif kind == MG_REC_EXP:
                out.append((step, "exp", limbs_to_word(q[k: k + 8]), limbs_to_word(q[k + 8: k + 16]), r))
                k += 16
            elif kind == MG_REC_HOOK:
                # (step, "hook", [stack[-1], stack[-2], ...], pc, opcode, fent)
                words = [r] + [limbs_to_word(q[k + 8 * j: k + 8 * j + 8]) for j in range(ln - 1)]
                k += 8 * (ln - 1)
                out.append((step, "hook", words, int(q[k]), int(q[k + 1]) & 0xFF, int(q[k + 2])))
                k += 3
            elif kind == MG_REC_SYMEXP:
                # (step, "symexp", Power node index)
                out.append((step, "symexp", int(q[k])))
                k += 1
            elif kind == MG_REC_SYMLEN:
                # (step, "symlen", the length's node index, 64)
                out.append((step, "symlen", int(q[k]), ln))
                k += 1
            elif kind == MG_REC_CDSIZE:
                # (step, "cdsize", the CODESIZE value pushed)
                out.append((step, "cdsize", r))
            elif kind == MG_REC_SYMKECCAK:
                # (step, "symkeccak", KECCAK node index, input bytes)
                out.append((step, "symkeccak", int(q[k]), ln))
                k += 1
            elif kind == MG_REC_ANNOT:
                # (step, "annot", atom, pc, opcode, post, stack[-1], stack[-2], fent)
                opw = int(q[k + 9])
                out.append((step, "annot", ln, int(q[k + 8]), opw & 0xFF, bool(opw & 0x100), r,
                            limbs_to_word(q[k: k + 8]), int(q[k + 10])))
                k += 11
            else:
                raise ValueError(f"lane {i}: bad record kind {kind} at word {k - MG_REC_HEADER}")
        return out

    def memory_bytes(self, i: int) -> bytes:
        return bytes(self.memory[i, : int(self.msize[i])])

    def return_data(self, i: int) -> Optional[bytes]:
        """RETURN/REVERT data: memory[off:off+len], bytes past msize read as 0
        (state/memory.py:152-157 reads missing keys as 0); None for a symbolic
        offset or length (MG_RET_SYMBOLIC)."""
        off, ln = int(self.ret_offset[i]), int(self.ret_len[i])
        if ln == MG_RET_SYMBOLIC:
            return None
        m = self.memory_bytes(i)
        return bytes(m[k] if k < len(m) else 0 for k in range(off, off + ln))

    def summary(self, i: int) -> dict:
        return {
            "status": STATUS_NAMES.get(int(self.status[i]), str(int(self.status[i]))),
            "aux": int(self.aux[i]), "pc": int(self.pc[i]), "sp": int(self.sp[i]),
            "msize": int(self.msize[i]), "depth": int(self.depth[i]),
            "steps": int(self.steps[i]),
            "gas": (int(self.gas_min[i]), int(self.gas_max[i])),
        }


# Fields compared lane-by-lane in parity tests (device vs oracle).
PARITY_SCALARS = ("pc", "sp", "msize", "depth", "status", "aux", "steps", "gas_min",
                  "gas_max", "storage_count", "trace_len", "rec_len", "fent")


def diff_batches(a: LaneBatch, b: LaneBatch, lanes: Optional[Iterable[int]] = None,
                 limit: int = 10) -> list:
    """Bit-exact comparison of two images; returns a list of human-readable diffs."""
    out = []
    idx = range(a.n) if lanes is None else lanes
    idx = np.asarray(list(idx))
    for f in PARITY_SCALARS:
        x, y = getattr(a, f)[idx], getattr(b, f)[idx]
        bad = np.nonzero(x != y)[0]
        for j in bad[:limit]:
            out.append(f"lane {idx[j]}: {f} {x[j]} != {y[j]}")
    # stack contents up to sp, memory up to msize, storage up to count, return data
    for i in idx:
        if len(out) >= limit:
            break
        sp = int(a.sp[i])
        if sp == int(b.sp[i]) and not np.array_equal(a.stack[i, :sp], b.stack[i, :sp]):
            out.append(f"lane {i}: stack differs")
        ms = int(a.msize[i])
        if ms == int(b.msize[i]) and not np.array_equal(a.memory[i, :ms], b.memory[i, :ms]):
            out.append(f"lane {i}: memory differs")
        if a.storage_dict(i, drop_zero=False) != b.storage_dict(i, drop_zero=False):
            out.append(f"lane {i}: storage differs")
        tl = int(a.trace_len[i])
        if a.shape.trace_cap and tl == int(b.trace_len[i]) and \
                not np.array_equal(a.trace[i, :tl], b.trace[i, :tl]):
            out.append(f"lane {i}: trace differs")
        rl = int(a.rec_len[i])
        if a.shape.rec_cap and rl == int(b.rec_len[i]) and \
                not np.array_equal(a.rec[i, :rl], b.rec[i, :rl]):
            out.append(f"lane {i}: function-manager records differ")
        if int(a.status[i]) in (MG_HALT_RETURN, MG_HALT_REVERT):
            if (a.ret_offset[i], a.ret_len[i]) != (b.ret_offset[i], b.ret_len[i]):
                out.append(f"lane {i}: return range differs")
    return out


_ALL_FIELDS = _U32_FIELDS + _U64_FIELDS + ("calldata", "env", "stack", "memory", "storage",
                                           "trace", "rec")


def bucket_order(batch: LaneBatch) -> np.ndarray:
    """Lane order that groups paths likely to run in lockstep: same code, same
    4-byte selector, same calldata length (SURVEY §7 'Divergence': bucket lanes
    by code and entry block).  Lanes are independent, so any order is correct;
    this one keeps a wave's 64 lanes on one instruction stream for longest."""
    sel = np.zeros(batch.n, dtype=np.uint64)
    for k in range(min(4, batch.shape.calldata_cap)):
        sel = (sel << np.uint64(8)) | batch.calldata[:, k].astype(np.uint64)
    return np.lexsort((batch.calldata_len, sel, batch.code_id))


def wave_aligned_order(batch: LaneBatch, selectors, wave: int = 64) -> np.ndarray:
    """bucket_order with every bucket of at least one wave starting and ending
    on a wave boundary.  A wave pays for the union of its lanes' paths (the
    longest C2 path, 203 steps, shared a wave with a 52-step bucket: 255 serial
    steps); the slack around a large bucket is filled with lanes whose calldata
    selects none of `selectors` (the code's dispatcher selectors,
    workloads.dispatch_selectors) -- calldata shorter than a selector first,
    then unknown selectors -- which take the dispatcher's fall-through, the
    shortest paths.  Still a permutation: parity is position independent."""
    base = bucket_order(batch)
    sel = np.zeros(batch.n, dtype=np.uint64)
    for k in range(min(4, batch.shape.calldata_cap)):
        sel = (sel << np.uint64(8)) | batch.calldata[:, k].astype(np.uint64)
    length = batch.calldata_len
    short = length < 4
    known = np.isin(sel, np.array(sorted(selectors), dtype=np.uint64)) & ~short
    fillers = np.concatenate([base[short[base]], base[(~known & ~short)[base]]])
    rest = base[known[base]]
    key = np.stack([batch.code_id[rest].astype(np.uint64), sel[rest],
                    length[rest].astype(np.uint64)], axis=1)
    cut = np.flatnonzero(np.any(key[1:] != key[:-1], axis=1)) + 1
    out, pos, f = [], 0, 0

    def pad():
        nonlocal pos, f
        k = min((-pos) % wave, len(fillers) - f)
        out.append(fillers[f:f + k])
        f += k
        pos += k
    for g in np.split(rest, cut):
        if len(g) >= wave:
            pad()
        out.append(g)
        pos += len(g)
        if len(g) >= wave:
            pad()
    out.append(fillers[f:])
    return np.concatenate(out)


def permuted(batch: LaneBatch, order: np.ndarray) -> LaneBatch:
    out = LaneBatch(batch.shape)
    for f in _ALL_FIELDS:
        getattr(out, f)[...] = getattr(batch, f)[order]
    return out
