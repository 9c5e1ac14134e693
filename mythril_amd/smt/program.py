"""Device formats of kernel 2: compiled constraint programs and candidate models.

A ``ProgramBatch`` is the host image of mg_dag_batch (include/mythgpu.h); a
``ModelPool`` the host image of mg_model_batch.  Instruction encoding matches
bv_eval.cuh (4 x u32: op | width<<8 | store<<17 | slot<<18, then three operand
refs kind<<30 | index, or immediates).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

OPS = ["copy", "bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod",
       "bvand", "bvor", "bvxor", "bvnot", "bvneg", "bvshl", "bvlshr", "bvashr",
       "eq", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
       "and", "or", "xor", "not", "implies", "ite", "extract", "concat", "zero_extend",
       "sign_extend", "bvadd_noovfl_u", "bvumul_noovfl", "bvsub_noudfl_u", "distinct"]
OPCODE = {name: i for i, name in enumerate(OPS)}
UNARY = {"copy", "bvnot", "bvneg", "not", "extract", "zero_extend", "sign_extend"}
REF_ACC, REF_SLOT, REF_VAR, REF_CONST = 0, 1, 2, 3
MAX_SLOTS = 8
TILE_INSNS = 2048


def ref(kind: int, idx: int) -> int:
    return (kind << 30) | idx


def enc_w0(op: str, width: int, store_slot: Optional[int] = None) -> int:
    w = OPCODE[op] | (width << 8)
    if store_slot is not None:
        w |= (1 << 17) | (store_slot << 18)
    return w


@dataclass
class ProgramBatch:
    insns: np.ndarray          # (total, 4) uint32
    prog_off: np.ndarray       # (n_dags + 1,) uint32
    consts: np.ndarray         # (n_consts, 8) uint32 little-endian limbs
    n_slots: int
    var_names: List[str] = field(default_factory=list)
    var_widths: List[int] = field(default_factory=list)

    @property
    def n_dags(self) -> int:
        return int(self.prog_off.shape[0] - 1)

    def program(self, d: int) -> np.ndarray:
        return self.insns[self.prog_off[d]:self.prog_off[d + 1]]

    def c_struct(self):
        from ..native import MgDagBatch
        self.insns = np.ascontiguousarray(self.insns, dtype=np.uint32)
        self.prog_off = np.ascontiguousarray(self.prog_off, dtype=np.uint32)
        self.consts = np.ascontiguousarray(self.consts, dtype=np.uint32)
        if self.consts.shape[0] == 0:
            self.consts = np.zeros((1, 8), dtype=np.uint32)
        s = MgDagBatch(self.n_dags, max(self.n_slots, 1), self.prog_off.ctypes.data,
                       self.insns.ctypes.data, self.consts.ctypes.data,
                       int(self.consts.shape[0]))
        return s


@dataclass
class ModelPool:
    """values[v, m] = value of variable v in model m (256-bit limbs), models in
    most-recently-used-first order (support_utils.py:62-63)."""
    values: np.ndarray         # (n_vars, n_models, 8) uint32

    @property
    def n_models(self) -> int:
        return int(self.values.shape[1])

    @property
    def n_vars(self) -> int:
        return int(self.values.shape[0])

    def c_struct(self):
        from ..native import MgModelBatch
        self.values = np.ascontiguousarray(self.values, dtype=np.uint32)
        return MgModelBatch(self.n_models, self.n_vars, self.values.ctypes.data)

    @staticmethod
    def from_dicts(models: List[Dict[str, int]], var_names: List[str], var_widths: List[int]):
        vals = np.zeros((max(len(var_names), 1), max(len(models), 1), 8), dtype=np.uint32)
        for m, model in enumerate(models):
            for v, (name, w) in enumerate(zip(var_names, var_widths)):
                x = model.get(name, 0) & ((1 << w) - 1)   # absent -> 0 (model completion)
                vals[v, m] = np.frombuffer(x.to_bytes(32, "little"), dtype="<u4")
        return ModelPool(vals)


def limbs(x: int) -> np.ndarray:
    return np.frombuffer((x & ((1 << 256) - 1)).to_bytes(32, "little"), dtype="<u4").copy()
