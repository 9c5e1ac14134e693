"""ctypes binding of libmythgpu.so (include/mythgpu.h).

The product path has exactly one implementation: the HIP library.  If the
shared object is missing or fails to load, ``load()`` raises — there is no CPU
fallback anywhere in ``mythril_amd`` (the CPU restatement under ``oracle/`` is
test infrastructure and is never imported here).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
LIB_PATH = PKG_DIR / "libmythgpu.so"
INCLUDE = PKG_DIR.parent / "include"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

MG_OK, MG_EINVAL, MG_EDEVICE, MG_ENOMEM, MG_ESTATE, MG_ENOCODE, MG_EUNSUPPORTED = 0, -1, -2, -3, -4, -5, -6


class MythGpuError(RuntimeError):
    pass


def sources():
    return sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cuh")) + sorted(CSRC.glob("*.h")) + [
        INCLUDE / "mythgpu.h"]


HASH_PATH = LIB_PATH.with_name(LIB_PATH.name + ".sha256")


def _command(out: str):
    # -structurizecfg-skip-uniform-regions: the interpreters' opcode switches
    # branch on wave-uniform values (readfirstlane); left unstructured they are
    # plain scalar branches instead of an exec-masked flag chain through every
    # case.  A/B on MI355X (scripts/archive/gpu_ab_skip.sh): kernel 2 C4 8.0 -> 11.9 G
    # constraint-evals/s (VGPRs 101 -> 69), kernel 1 C2 36.6 -> 38.4 G lane-steps/s.
    return [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17",
            "-mllvm", "-structurizecfg-skip-uniform-regions=true",
            "-Wno-unused-value", "-Wno-unused-result", str(CSRC / "mythgpu.hip"), "-o", out]


def source_hash() -> str:
    """sha256 over the sources and the compile command: the identity of a build."""
    import hashlib
    h = hashlib.sha256()
    for p in sources():
        h.update(p.name.encode() + b"\0" + p.read_bytes() + b"\0")
    # the flags only: the compiler and source paths differ between this container
    # and the GPU box's copy of the tree
    h.update(" ".join(a for a in _command("OUT")[1:] if not a.startswith("/")).encode())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile libmythgpu.so for gfx950 in-tree (hipcc; one translation unit).
    Rebuilds whenever the recorded source hash differs (a library copied from
    elsewhere, or built from older sources, is never trusted by mtime)."""
    want = source_hash()
    if not force and LIB_PATH.exists() and HASH_PATH.exists() and \
            HASH_PATH.read_text().strip() == want:
        return LIB_PATH
    cmd = _command(str(LIB_PATH) + ".tmp")
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(str(LIB_PATH) + ".tmp", LIB_PATH)
    HASH_PATH.write_text(want + "\n")
    return LIB_PATH


class MgStepStats(ctypes.Structure):
    _fields_ = [("lane_steps", ctypes.c_uint64), ("running", ctypes.c_uint32),
                ("halted", ctypes.c_uint32), ("hooked", ctypes.c_uint32),
                ("escaped", ctypes.c_uint32), ("kernel_ms", ctypes.c_float),
                ("launches", ctypes.c_uint32)]


class MgBatchCfg(ctypes.Structure):
    _fields_ = [("n_lanes", ctypes.c_uint32), ("stack_cap", ctypes.c_uint32),
                ("mem_cap", ctypes.c_uint32), ("calldata_cap", ctypes.c_uint32),
                ("storage_cap", ctypes.c_uint32), ("coverage", ctypes.c_uint32),
                ("trace_cap", ctypes.c_uint32), ("rec_cap", ctypes.c_uint32)]


class MgDagBatch(ctypes.Structure):
    _fields_ = [("n_dags", ctypes.c_uint32), ("n_slots", ctypes.c_uint32),
                ("prog_off", ctypes.c_void_p), ("insns", ctypes.c_void_p),
                ("consts", ctypes.c_void_p), ("n_consts", ctypes.c_uint32)]


class MgModelBatch(ctypes.Structure):
    _fields_ = [("n_models", ctypes.c_uint32), ("n_vars", ctypes.c_uint32),
                ("values", ctypes.c_void_p), ("n_tables", ctypes.c_uint32),
                ("tab_start", ctypes.c_void_p), ("tab_count", ctypes.c_void_p),
                ("tab_entries", ctypes.c_void_p), ("n_entries", ctypes.c_uint32),
                ("tab_default", ctypes.c_void_p)]


# every symbol include/mythgpu.h declares: name -> (restype, argtypes)
_P, _U32, _U64, _I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
_PU32 = ctypes.POINTER(ctypes.c_uint32)
SIGNATURES = {
    "mg_abi_version": (_I, []),
    "mg_cc_open": (_I, [ctypes.POINTER(_P)]),
    "mg_cc_close": (None, [_P]),
    "mg_cc_error": (ctypes.c_char_p, [_P]),
    "mg_cc_add": (_I, [_P, _P, _U32, _P, _U32, _P]),
    "mg_cc_compile": (_I, [_P, _U32, _P, _U32, _PU32, _PU32]),
    "mg_open": (_I, [_I, ctypes.POINTER(_P)]),
    "mg_close": (None, [_P]),
    "mg_last_error": (ctypes.c_char_p, [_P]),
    "mg_opcode_info": (_I, [_U32, _PU32, _PU32, _PU32]),
    "mg_load_code": (_I, [_P, ctypes.c_char_p, ctypes.c_size_t, _PU32]),
    "mg_code_info": (_I, [_P, _U32, _PU32]),
    "mg_code_fentries": (_I, [_P, _U32, _P, _U32]),
    "mg_code_table": (_I, [_P, _U32, _P, _P, _U32]),
    "mg_lanes_alloc": (_I, [_P, ctypes.POINTER(MgBatchCfg)]),
    "mg_lanes_upload": (_I, [_P, _P, _U32, _U32]),
    "mg_lanes_download": (_I, [_P, _P, _U32, _U32]),
    "mg_lanes_download_live": (_I, [_P, _P, _U32, _U32]),
    "mg_lanes_upload_live": (_I, [_P, _P, _U32, _U32]),
    "mg_lanes_reset": (_I, [_P]),
    "mg_step": (_I, [_P, _P, _U32, _U32, ctypes.POINTER(MgStepStats)]),
    "mg_step_async": (_I, [_P, _P, _U32, _U32]),
    "mg_run_batches": (_I, [_P, _P, _U32, _U32, _U32, ctypes.POINTER(MgStepStats)]),
    "mg_step_until": (_I, [_P, _P, _U32, _U32, _U32, ctypes.POINTER(MgStepStats)]),
    "mg_set_loop_bound": (_I, [_P, _U32]),
    "mg_eval_bits": (_I, [_P, ctypes.POINTER(MgDagBatch), ctypes.POINTER(MgModelBatch), _P, _P, _P,
                          ctypes.POINTER(ctypes.c_float)]),
    "mg_step_profile": (_I, [_P, _P, _U32, _U32, _P, _P]),
    "mg_sync": (_I, [_P]),
    "mg_coverage": (_I, [_P, _U32, _P, _U32]),
    "mg_coverage_clear": (_I, [_P]),
    "mg_event_counts": (_I, [_P, _P, _P, _U32, _U32]),
    "mg_eval": (_I, [_P, ctypes.POINTER(MgDagBatch), ctypes.POINTER(MgModelBatch), _P, _P,
                     ctypes.POINTER(ctypes.c_float)]),
    "mg_eval_upload": (_I, [_P, ctypes.POINTER(MgDagBatch), ctypes.POINTER(MgModelBatch)]),
    "mg_eval_run": (_I, [_P, _U32, _U32, ctypes.POINTER(ctypes.c_float)]),
    "mg_eval_download": (_I, [_P, _P, _P, _U32, _U32]),
    "mg_sym_alloc": (_I, [_P, _U32, _U32]),
    "mg_sym_upload": (_I, [_P, _P, _U32, _U32]),
    "mg_sym_download": (_I, [_P, _P, _U32, _U32]),
    "mg_taint_alloc": (_I, [_P, _U32]),
    "mg_taint_program": (_I, [_P, _P]),
    "mg_taint_force": (_I, [_P, _U32, _P, _U32]),
    "mg_taint_upload": (_I, [_P, _P, _U32, _U32]),
    "mg_taint_download": (_I, [_P, _P, _U32, _U32]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load the in-tree libmythgpu.so; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("MYTHGPU_LIB", LIB_PATH))   # A/B runs point this at a variant
    if not path.exists():
        raise MythGpuError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback in mythril_amd)")
    if "MYTHGPU_LIB" not in os.environ:
        got = HASH_PATH.read_text().strip() if HASH_PATH.exists() else "missing"
        if got != source_hash():
            raise MythGpuError(
                f"{path} was not built from the current sources (recorded hash {got[:12]}): "
                "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
