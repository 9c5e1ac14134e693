"""ctypes front end of the C oracle stepper (oracle/evm_ref.c) — TEST INFRASTRUCTURE ONLY."""
import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import lib


def keccak256(data: bytes, pad: int = 0x01) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().orc_keccak256_pad(bytes(data), len(data), pad, out)
    return out.raw


def opcode_info(byte: int):
    g0, g1, r = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    rc = lib().orc_opcode_info(byte, ctypes.byref(g0), ctypes.byref(g1), ctypes.byref(r))
    return None if rc else (g0.value, g1.value, r.value)


class OracleEVM:
    """Loaded codes + a run() over a mythril_amd.lanes.LaneBatch image."""

    def __init__(self):
        lib().orc_reset_codes()
        self.codes: List[bytes] = []

    def load_code(self, code: bytes) -> int:
        cid = ctypes.c_uint32()
        if lib().orc_load_code(bytes(code), len(code), ctypes.byref(cid)):
            raise RuntimeError("oracle: too many codes")
        self.codes.append(bytes(code))
        return cid.value

    def code_table(self, code_id: int):
        n = ctypes.c_uint32()
        lib().orc_code_info(code_id, ctypes.byref(n), None, None)
        ops = np.zeros(n.value, dtype=np.uint8)
        addrs = np.zeros(n.value, dtype=np.uint32)
        lib().orc_code_info(code_id, ctypes.byref(n), ops.ctypes.data, addrs.ctypes.data)
        return ops, addrs

    def code_fentries(self, code_id: int) -> np.ndarray:
        """uint8[n_instr]: 1 where a JUMP / JUMPI landing switches the function
        name (the oracle's own restatement of the dispatcher table)."""
        ops, _ = self.code_table(code_id)
        out = np.zeros(ops.size, dtype=np.uint8)
        lib().orc_code_fentries(code_id, out.ctypes.data)
        return out

    def set_coverage(self, code_id: int, buf: Optional[np.ndarray]) -> None:
        """Record into `buf` (uint8[n_instr], kept alive by the caller) the
        instructions lanes of `code_id` start, as the device's mg_coverage."""
        if buf is not None:
            assert buf.dtype == np.uint8 and buf.flags.c_contiguous
        lib().orc_set_coverage(code_id, None if buf is None else buf.ctypes.data)

    def run(self, batch, first: int = 0, n: Optional[int] = None,
            hook_mask: Sequence[int] = (0, 0, 0, 0), max_steps: int = 1 << 30,
            max_depth: int = 0, horizon: int = 0, loop_bound: int = 0) -> int:
        n = batch.n - first if n is None else n
        mask = (ctypes.c_uint64 * 4)(*[int(x) for x in hook_mask])
        soa = batch.soa()
        return int(lib().orc_run_loop(ctypes.addressof(soa), first, n, mask, max_steps, max_depth,
                                      horizon, loop_bound))


def loop_count(trace) -> int:
    """oracle/evm_ref.c orc_loop_count (literal get_loop_count)."""
    arr = np.ascontiguousarray(np.asarray(trace, dtype=np.uint32))
    return int(lib().orc_loop_count(arr.ctypes.data, arr.size))
