"""Test-only stand-in for mythril_amd.device.GpuDevice backed by the C oracle
(oracle/evm_ref.c), so the host LASER mirror (mythril_amd/laser) and the
multi-rank drivers run end to end on CPU under `-m "not gpu"` (gloo ranks).

It is test infrastructure: the product path (LaserEVM's default device) is
GpuDevice, which fails loudly without libmythgpu.so.  Lane images live in a
host LaneBatch; `step` is one oracle run over it with the launch's hook mask,
step budget, depth cut, horizon and loop bound, so its results are the ones the
GPU parity tests pin kernel 1 against.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from mythril_amd.device import StepStats
from mythril_amd.lanes import (_ALL_FIELDS, _SYM_FIELDS, _TAINT_FIELDS, LaneBatch, MG_DEPTH, MG_ESC_SYMBOLIC,
                               MG_ESCAPE, MG_FORK, MG_HALT_END, MG_HOOK, MG_LANE_HOOK_ACK, MG_LANE_SYMBOLIC,
                               MG_LANE_TAINT, MG_RUNNING)
from oracle.evm_ref import OracleEVM

from taintref import run_lane


class OracleDevice:
    def __init__(self):
        self.o = OracleEVM()
        self.codes = []
        self._cov: Dict[int, np.ndarray] = {}
        self._cov_on = False
        self._img: Optional[LaneBatch] = None
        self._bound = 0
        self.shape = None
        self._actions = np.zeros(256, dtype=np.uint32)
        self._force = {}

    # -- codes
    def load_code(self, code: bytes) -> int:
        cid = self.o.load_code(bytes(code))
        self.codes.append(bytes(code))
        ops, _ = self.o.code_table(cid)
        self._cov[cid] = np.zeros(max(ops.size, 1), dtype=np.uint8)
        return cid

    def n_instr(self, code_id: int) -> int:
        ops, _ = self.o.code_table(code_id)
        return int(ops.size)

    # -- lanes
    def alloc(self, shape, coverage: bool = False):
        self.shape = shape
        self._img = LaneBatch(shape)
        self._cov_on = bool(coverage)

    def set_taint_program(self, actions):
        self._actions = np.asarray(actions, dtype=np.uint32).reshape(256).copy()

    def set_taint_force(self, code_id, flags):
        self._force[int(code_id)] = np.asarray(flags, dtype=np.uint8).copy()

    def _copy(self, src: LaneBatch, dst: LaneBatch, first: int, n: int):
        fields = _ALL_FIELDS + (_SYM_FIELDS if src.symbolic and dst.symbolic else ()) + (
            _TAINT_FIELDS if src.taint and dst.taint else ())
        for f in fields:
            a, b = getattr(dst, f), getattr(src, f)
            if a.shape[1:] == b.shape[1:]:
                a[first:first + n] = b[first:first + n]
            else:                      # slim image (workloads.slim_copy): the overlap, rest zero
                a[first:first + n] = 0
                sl = tuple(slice(0, min(x, y)) for x, y in zip(a.shape[1:], b.shape[1:]))
                a[(slice(first, first + n),) + sl] = b[(slice(first, first + n),) + sl]

    def upload(self, batch: LaneBatch, first: int = 0):
        self._copy(batch, self._img, first, batch.n)
        self._init = LaneBatch(self._img.shape)           # the resident initial image
        self._copy(self._img, self._init, 0, self._img.n)

    def reset(self):
        self._copy(self._init, self._img, 0, self._img.n)

    def run_batches(self, n_batches: int, hook_mask=None, max_steps: int = 1 << 30,
                    max_depth: int = 0):
        """mg_run_batches: n x (reset from the resident image + one step)."""
        out = []
        for _ in range(n_batches):
            self.reset()
            out.append(self.step(hook_mask, max_steps, max_depth))
        return out

    def download(self, batch: LaneBatch, first: int = 0):
        self._copy(self._img, batch, first, batch.n)

    def upload_range(self, batch: LaneBatch, first: int, n: int, live: bool = False):
        self._copy(batch, self._img, first, n)

    def download_range(self, batch: LaneBatch, first: int, n: int, live: bool = False):
        self._copy(self._img, batch, first, n)

    def set_loop_bound(self, bound: int):
        self._bound = int(bound)

    def step(self, hook_mask=None, max_steps: int = 1 << 30, max_depth: int = 0,
             horizon: int = 0) -> StepStats:
        for cid, buf in self._cov.items():
            self.o.set_coverage(cid, buf if self._cov_on else None)
        bound = self._bound if self._img.shape.trace_cap else 0
        self._park_symbolic(hook_mask, max_depth, bound)
        img = self._img
        # taint lanes are k_sym_step's: the restatement steps them (tests/taintref.py)
        tl = np.nonzero((img.status == MG_RUNNING) & ((img.flags & MG_LANE_TAINT) != 0)
                        & ((img.flags & MG_LANE_SYMBOLIC) == 0))[0] if img.taint else np.zeros(0, dtype=int)
        img.status[tl] = 0xFF
        steps = self.o.run(img, hook_mask=hook_mask or (0, 0, 0, 0), max_steps=max_steps,
                           max_depth=max_depth, horizon=horizon, loop_bound=bound)
        img.status[tl] = MG_RUNNING
        mask = hook_mask or (0, 0, 0, 0)
        for i in tl:
            ops, _ = self.o.code_table(int(img.code_id[i]))
            steps += run_lane(self.o, ops, img, int(i), self._actions, mask, max_steps, max_depth, horizon, bound,
                              self._force.get(int(img.code_id[i])))
        for cid in self._cov:
            self.o.set_coverage(cid, None)
        s = self._img.status
        return StepStats(steps, int((s == MG_RUNNING).sum()),
                         int(((s != MG_RUNNING) & (s != MG_HOOK) & (s != MG_ESCAPE)).sum()),
                         int((s == MG_HOOK).sum()), int((s == MG_ESCAPE).sum()), 0.0)

    def _park_symbolic(self, hook_mask, max_depth, bound: int = 0):
        """The oracle has no symbolic lanes: a running MG_LANE_SYMBOLIC lane stops
        before its next instruction exactly as k_sym_step stops before one it
        cannot run (depth cut, past the end, the instruction traced and the loop
        bound checked, hook, else MG_ESC_SYMBOLIC), so the host's escape handler
        executes it (test stand-in for k_sym_step)."""
        img = self._img
        live = np.nonzero((img.status == MG_RUNNING) & ((img.flags & MG_LANE_SYMBOLIC) != 0))[0]
        mask = hook_mask or (0, 0, 0, 0)
        for i in live:
            ops, _ = self.o.code_table(int(img.code_id[i]))
            pc = int(img.pc[i])
            if max_depth and int(img.depth[i]) >= max_depth:
                img.status[i] = MG_DEPTH
            elif pc >= ops.size:
                img.status[i] = MG_HALT_END
            else:
                op = int(ops[pc])
                acked = int(img.flags[i]) & MG_LANE_HOOK_ACK
                if bound and not acked:
                    # BoundedLoopsStrategy sees every instruction the path is popped
                    # at (sym_step.cuh: trace_step before the hook / escape checks):
                    # the oracle traces it and stops there (a probe hook on it)
                    probe = [int(x) for x in mask]
                    probe[op >> 6] |= 1 << (op & 63)
                    self.o.run(img, int(i), 1, hook_mask=probe, max_steps=1, max_depth=max_depth,
                               loop_bound=bound)
                    if int(img.status[i]) != MG_HOOK:
                        continue                # the loop bound, or a full trace: as the device
                    img.status[i], img.aux[i] = MG_RUNNING, 0
                hooked = (int(mask[op >> 6]) >> (op & 63)) & 1 and not acked
                sp = int(img.sp[i])
                fork = (op == 0x57 and not hooked and sp >= 2 and img.symbolic and int(img.stag[i, sp - 2])
                        and not int(img.stag[i, sp - 1]))
                if fork:                        # k_sym_step: a JUMPI on a symbolic condition
                    img.status[i], img.aux[i] = MG_FORK, op
                    continue
                img.status[i] = MG_HOOK if hooked else MG_ESCAPE
                img.aux[i] = op if hooked else op | (MG_ESC_SYMBOLIC << 8)

    # -- coverage
    def coverage(self, code_id: int) -> np.ndarray:
        return self._cov[code_id][:self.n_instr(code_id)].copy()

    def coverage_clear(self):
        for buf in self._cov.values():
            buf[:] = 0


class OracleK2:
    """Test stand-in for kernel 2's entry points (mg_eval / mg_eval_bits),
    backed by the C evaluator oracle/bv_ref.c."""

    def __init__(self):
        self.launches = 0

    def eval(self, prog, pool):
        from oracle.bv_ref import eval_batch
        self.launches += 1
        fs, sc = eval_batch(prog, pool)
        return fs, sc, 0.0

    def eval_bits(self, prog, pool):
        from oracle.bv_ref import eval_batch
        self.launches += 1
        n, m = prog.n_dags, pool.n_models
        bits = np.zeros((n, (m + 63) // 64), dtype=np.uint64)
        fs, sc = eval_batch(prog, pool, bits=bits)
        return fs, sc, bits, 0.0
