"""ctypes front end of the C program evaluator (oracle/bv_ref.c) — TEST INFRASTRUCTURE ONLY."""
import ctypes
import os

import numpy as np

from . import lib


def eval_batch(prog, models, first: int = 0, count: int = None, threads: int = 0, bits=None):
    """(first_sat, sat_count) of programs [first, first+count) over every model;
    `bits` (uint64 [n_dags][ceil(n_models / 64)], zeroed) also receives each
    program's per-model satisfaction bitmap."""
    n = prog.n_dags
    count = n - first if count is None else count
    from .cpu_baseline import _cpu_share
    threads = threads or _cpu_share()
    fs = np.zeros(n, dtype=np.uint32)
    sc = np.zeros(n, dtype=np.uint32)
    insns = np.ascontiguousarray(prog.insns, dtype=np.uint32)
    off = np.ascontiguousarray(prog.prog_off, dtype=np.uint32)
    consts = np.ascontiguousarray(prog.consts if prog.consts.size else np.zeros((1, 8)), dtype=np.uint32)
    vals = np.ascontiguousarray(models.values, dtype=np.uint32)
    f = lib().orb_eval_tab_bits
    f.restype = None
    f.argtypes = ([ctypes.c_void_p] * 4 + [ctypes.c_uint32] * 5 + [ctypes.c_void_p] * 2 +
                  [ctypes.c_uint32, ctypes.c_uint32] + [ctypes.c_void_p] * 5)
    if models.n_tables:
        ts, tc, te, td = (np.ascontiguousarray(x, dtype=np.uint32) for x in
                          (models.tab_start, models.tab_count,
                           models.tab_entries if models.tab_entries.size else np.zeros((1, 32)),
                           models.tab_default))
        tabs = (models.n_tables, ts.ctypes.data, tc.ctypes.data, te.ctypes.data, td.ctypes.data)
    else:
        tabs = (0, None, None, None, None)
    f(insns.ctypes.data, off.ctypes.data, consts.ctypes.data, vals.ctypes.data, models.n_vars,
      models.n_models, prog.n_slots, first, count, fs.ctypes.data, sc.ctypes.data, threads, *tabs,
      None if bits is None else bits.ctypes.data)
    return fs[first:first + count], sc[first:first + count]
