"""One MI355X context: codes, a resident lane batch, stepping and evaluation.

Thin object wrapper over the C-ABI (native.py).  One ``GpuDevice`` per GPU and
per process (contexts are single-threaded; multi-GPU = one
process per GPU).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import native
from .lanes import LaneBatch, LaneShape


@dataclass
class StepStats:
    lane_steps: int
    running: int
    halted: int
    hooked: int
    escaped: int
    kernel_ms: float


def _mask_array(hook_mask: Optional[Sequence[int]]):
    m = list(hook_mask) if hook_mask is not None else [0, 0, 0, 0]
    return (ctypes.c_uint64 * 4)(*[int(x) & ((1 << 64) - 1) for x in m])


def hook_mask_for(opcodes) -> list:
    """256-bit mask (4 x u64) with the given opcode bytes set."""
    m = [0, 0, 0, 0]
    for b in opcodes:
        m[b >> 6] |= 1 << (b & 63)
    return m


class GpuDevice:
    def __init__(self, device: int = 0):
        self.lib = native.load()
        self.ctx = ctypes.c_void_p()
        rc = self.lib.mg_open(device, ctypes.byref(self.ctx))
        if rc != native.MG_OK:
            raise native.MythGpuError(f"mg_open({device}) failed with {rc}")
        self.device = device
        self.shape: Optional[LaneShape] = None
        self.codes = []

    # -- errors --------------------------------------------------------------
    def _check(self, rc: int, what: str):
        if rc != native.MG_OK:
            msg = self.lib.mg_last_error(self.ctx)
            raise native.MythGpuError(f"{what}: rc={rc}: {msg.decode() if msg else ''}")

    def close(self):
        if self.ctx:
            self.lib.mg_close(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- codes ---------------------------------------------------------------
    def load_code(self, code: bytes) -> int:
        cid = ctypes.c_uint32()
        self._check(self.lib.mg_load_code(self.ctx, bytes(code), len(code), ctypes.byref(cid)),
                    "mg_load_code")
        self.codes.append(bytes(code))
        return cid.value

    def n_instr(self, code_id: int) -> int:
        n = ctypes.c_uint32()
        self._check(self.lib.mg_code_info(self.ctx, code_id, ctypes.byref(n)), "mg_code_info")
        return n.value

    def code_fentries(self, code_id: int) -> np.ndarray:
        """mg_code_fentries: uint8[n_instr], bit 0 = a JUMP / JUMPI landing here
        switches active_function_name, bit 1 = the same for the next index."""
        out = np.zeros(self.n_instr(code_id), dtype=np.uint8)
        self._check(self.lib.mg_code_fentries(self.ctx, code_id, out.ctypes.data, out.size), "mg_code_fentries")
        return out

    def code_table(self, code_id: int):
        """mg_code_table: (opcode byte per instruction, byte address per instruction)."""
        n = self.n_instr(code_id)
        ops = np.zeros(n, dtype=np.uint8)
        addrs = np.zeros(n, dtype=np.uint32)
        self._check(self.lib.mg_code_table(self.ctx, code_id, ops.ctypes.data, addrs.ctypes.data, n),
                    "mg_code_table")
        return ops, addrs

    # -- lanes ---------------------------------------------------------------
    def alloc(self, shape: LaneShape, coverage: bool = False):
        cfg = native.MgBatchCfg(shape.n, shape.stack_cap, shape.mem_cap, shape.calldata_cap,
                                shape.storage_cap, 1 if coverage else 0, shape.trace_cap,
                                shape.rec_cap)
        self._check(self.lib.mg_lanes_alloc(self.ctx, ctypes.byref(cfg)), "mg_lanes_alloc")
        if shape.node_cap:
            self._check(self.lib.mg_sym_alloc(self.ctx, shape.node_cap, max(shape.const_cap, 1)),
                        "mg_sym_alloc")
        if shape.obj_cap:
            self._check(self.lib.mg_taint_alloc(self.ctx, shape.obj_cap), "mg_taint_alloc")
        self.shape = shape

    def set_taint_program(self, actions) -> None:
        """mg_taint_program: the per-opcode action words of the batch-safe hooks
        (256 x uint32, mythril_amd/laser/taint.py)."""
        arr = np.ascontiguousarray(np.asarray(actions, dtype=np.uint32).reshape(256))
        self._check(self.lib.mg_taint_program(self.ctx, arr.ctypes.data), "mg_taint_program")

    def set_taint_force(self, code_id: int, flags) -> None:
        """mg_taint_force: instructions of a code where taint lanes stop for the
        host instead of applying the batch-safe actions."""
        arr = np.ascontiguousarray(np.asarray(flags, dtype=np.uint8))
        self._check(self.lib.mg_taint_force(self.ctx, int(code_id), arr.ctypes.data, arr.size),
                    "mg_taint_force")

    def _planes(self, batch: LaneBatch, first: int, n: int, up: bool, dev_first: Optional[int] = None):
        """Symbolic / taint planes of host lanes [first, first + n) to or from
        device lanes [dev_first, dev_first + n) (dev_first defaults to first)."""
        d = first if dev_first is None else dev_first
        if batch.symbolic:
            s = batch.sym_soa_range(first, n)
            fn = self.lib.mg_sym_upload if up else self.lib.mg_sym_download
            self._check(fn(self.ctx, ctypes.addressof(s), d, n), "mg_sym_upload" if up else "mg_sym_download")
        if batch.taint:
            t = batch.taint_soa_range(first, n)
            fn = self.lib.mg_taint_upload if up else self.lib.mg_taint_download
            self._check(fn(self.ctx, ctypes.addressof(t), d, n),
                        "mg_taint_upload" if up else "mg_taint_download")

    def upload(self, batch: LaneBatch, first: int = 0):
        soa = batch.soa()
        self._check(self.lib.mg_lanes_upload(self.ctx, ctypes.addressof(soa), first, batch.n),
                    "mg_lanes_upload")
        self._planes(batch, 0, batch.n, True, first)

    def download(self, batch: LaneBatch, first: int = 0):
        soa = batch.soa()
        self._check(self.lib.mg_lanes_download(self.ctx, ctypes.addressof(soa), first, batch.n),
                    "mg_lanes_download")
        self._planes(batch, 0, batch.n, False, first)

    def upload_range(self, batch: LaneBatch, first: int, n: int, live: bool = False):
        """Upload lanes [first, first + n) of `batch` to the same device lanes.
        live=True: only what a step reads, below the range's largest sp /
        msize / storage count / record and trace length (mg_lanes_upload_live)."""
        soa = batch.soa_range(first, n)
        fn = self.lib.mg_lanes_upload_live if live else self.lib.mg_lanes_upload
        self._check(fn(self.ctx, ctypes.addressof(soa), first, n),
                    "mg_lanes_upload_live" if live else "mg_lanes_upload")
        self._planes(batch, first, n, True)

    def download_range(self, batch: LaneBatch, first: int, n: int, live: bool = False):
        """Download lanes [first, first + n).  live=True (the host image was
        uploaded from `batch`): only what a step can have changed, below the
        range's largest sp / msize / storage count / record length
        (mg_lanes_download_live)."""
        soa = batch.soa_range(first, n)
        fn = self.lib.mg_lanes_download_live if live else self.lib.mg_lanes_download
        self._check(fn(self.ctx, ctypes.addressof(soa), first, n),
                    "mg_lanes_download_live" if live else "mg_lanes_download")
        self._planes(batch, first, n, False)

    def set_loop_bound(self, bound: int):
        """BoundedLoopsStrategy on the device (0 = off); needs trace_cap > 0."""
        self._check(self.lib.mg_set_loop_bound(self.ctx, int(bound)), "mg_set_loop_bound")

    def reset(self):
        self._check(self.lib.mg_lanes_reset(self.ctx), "mg_lanes_reset")

    def step(self, hook_mask=None, max_steps: int = 1 << 30, max_depth: int = 0,
             horizon: int = 0) -> StepStats:
        """mg_step (horizon 0) or mg_step_until: lanes also pause once their
        cumulative steps reach `horizon`."""
        st = native.MgStepStats()
        if horizon:
            rc = self.lib.mg_step_until(self.ctx, _mask_array(hook_mask), max_steps, max_depth,
                                        horizon, ctypes.byref(st))
        else:
            rc = self.lib.mg_step(self.ctx, _mask_array(hook_mask), max_steps, max_depth,
                                  ctypes.byref(st))
        self._check(rc, "mg_step")
        return StepStats(st.lane_steps, st.running, st.halted, st.hooked, st.escaped, st.kernel_ms)

    def run_batches(self, n_batches: int, hook_mask=None, max_steps: int = 1 << 30,
                    max_depth: int = 0):
        """mg_run_batches: n_batches x (reset from the resident image + one
        stepping launch) enqueued back to back, one host wait; per-batch stats."""
        st = (native.MgStepStats * n_batches)()
        self._check(self.lib.mg_run_batches(self.ctx, _mask_array(hook_mask), max_steps, max_depth,
                                            n_batches, st), "mg_run_batches")
        return [StepStats(s.lane_steps, s.running, s.halted, s.hooked, s.escaped, s.kernel_ms)
                for s in st]

    def step_profile(self, hook_mask=None, max_steps: int = 1 << 30, max_depth: int = 0):
        """Step with per-opcode counters; returns (op_counts[256], extra[4])."""
        ops = np.zeros(256, dtype=np.uint64)
        extra = np.zeros(4, dtype=np.uint64)
        self._check(self.lib.mg_step_profile(self.ctx, _mask_array(hook_mask), max_steps, max_depth,
                                             ops.ctypes.data, extra.ctypes.data), "mg_step_profile")
        return ops, extra

    def step_async(self, hook_mask=None, max_steps: int = 1 << 30, max_depth: int = 0):
        self._check(self.lib.mg_step_async(self.ctx, _mask_array(hook_mask), max_steps, max_depth),
                    "mg_step_async")

    def sync(self):
        self._check(self.lib.mg_sync(self.ctx), "mg_sync")

    def coverage(self, code_id: int) -> np.ndarray:
        n = self.n_instr(code_id)
        out = np.zeros(max(n, 1), dtype=np.uint8)
        self._check(self.lib.mg_coverage(self.ctx, code_id, out.ctypes.data, out.size), "mg_coverage")
        return out[:n]

    def coverage_clear(self):
        self._check(self.lib.mg_coverage_clear(self.ctx), "mg_coverage_clear")

    def event_counts(self, n: int, first: int = 0):
        sha3 = np.zeros(n, dtype=np.uint32)
        exp = np.zeros(n, dtype=np.uint32)
        self._check(self.lib.mg_event_counts(self.ctx, sha3.ctypes.data, exp.ctypes.data, first, n),
                    "mg_event_counts")
        return sha3, exp

    # -- kernel 2 ------------------------------------------------------------
    def eval_upload(self, program, models):
        """program: mythril_amd.smt.program.ProgramBatch; models: ModelPool."""
        self._dags = program.c_struct()
        self._models = models.c_struct()
        self._check(self.lib.mg_eval_upload(self.ctx, ctypes.byref(self._dags),
                                            ctypes.byref(self._models)), "mg_eval_upload")
        self._n_dags = program.n_dags

    def eval_run(self, first: int = 0, count: Optional[int] = None) -> float:
        count = self._n_dags - first if count is None else count
        ms = ctypes.c_float()
        self._check(self.lib.mg_eval_run(self.ctx, first, count, ctypes.byref(ms)), "mg_eval_run")
        return ms.value

    def eval_download(self, first: int = 0, count: Optional[int] = None):
        count = self._n_dags - first if count is None else count
        fs = np.zeros(count, dtype=np.uint32)
        sc = np.zeros(count, dtype=np.uint32)
        self._check(self.lib.mg_eval_download(self.ctx, fs.ctypes.data, sc.ctypes.data, first, count),
                    "mg_eval_download")
        return fs, sc

    def eval_bits(self, program, models):
        """(first_sat, sat_count, sat_bits[n_dags, ceil(n_models/64)] uint64, ms)."""
        dags, mods = program.c_struct(), models.c_struct()
        n, words = program.n_dags, (models.n_models + 63) // 64
        fs = np.zeros(n, dtype=np.uint32)
        sc = np.zeros(n, dtype=np.uint32)
        bits = np.zeros((n, words), dtype=np.uint64)
        ms = ctypes.c_float()
        self._check(self.lib.mg_eval_bits(self.ctx, ctypes.byref(dags), ctypes.byref(mods),
                                          fs.ctypes.data, sc.ctypes.data, bits.ctypes.data,
                                          ctypes.byref(ms)), "mg_eval_bits")
        return fs, sc, bits, ms.value

    def eval(self, program, models):
        self.eval_upload(program, models)
        ms = self.eval_run()
        fs, sc = self.eval_download()
        return fs, sc, ms
