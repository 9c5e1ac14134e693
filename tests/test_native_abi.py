"""CPU-side checks of the C-ABI library (no GPU needed): it loads, exports every
symbol include/mythgpu.h declares, and its opcode table matches the reference's."""
import re
from pathlib import Path

from mythril_amd import native
from vmtests_util import load_json

HEADER = Path(__file__).resolve().parent.parent / "include" / "mythgpu.h"


def declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(mg_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = native.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(native.SIGNATURES), set(syms) ^ set(native.SIGNATURES)
    assert lib.mg_abi_version() == 15


def test_device_opcode_table_matches_reference():
    import ctypes
    lib = native.load()
    table = load_json("opcodes.json")
    by_byte = {d["byte"]: d for d in table.values()}
    g0, g1, r = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    for byte in range(256):
        rc = lib.mg_opcode_info(byte, ctypes.byref(g0), ctypes.byref(g1), ctypes.byref(r))
        if byte not in by_byte:
            assert rc == -1, hex(byte)
        else:
            d = by_byte[byte]
            assert rc == 0 and (g0.value, g1.value, r.value) == (d["gas"][0], d["gas"][1],
                                                                d["stack"][0]), hex(byte)


def test_open_without_gpu_fails_cleanly():
    import ctypes
    import torch
    if torch.cuda.is_available():
        return
    lib = native.load()
    ctx = ctypes.c_void_p()
    assert lib.mg_open(0, ctypes.byref(ctx)) != 0


def test_exact_library_exports_every_declared_symbol():
    """include/mythsmt.h (the exact procedure behind kernel 2): libmythsmt.so
    loads, exports every declared function with the binding's signature, and
    its opcode numbering is exact.py's."""
    from mythril_amd.smt import exact
    text = (HEADER.parent / "mythsmt.h").read_text()
    syms = sorted(set(re.findall(r"\b(ms_[a-z_0-9]+)\s*\(", text)))
    lib = exact.load()
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(exact.SIGNATURES), set(syms) ^ set(exact.SIGNATURES)
    assert lib.ms_abi_version() == 1
    enum = re.search(r"enum \{(.*?)\};", text, re.S).group(1)
    names = [n.strip() for n in re.findall(r"MS_([A-Z_0-9]+)", enum) if n != "N_OPS"]
    assert [n.lower() for n in names] == [k.lower() for k in sorted(exact.OPS, key=exact.OPS.get)]
