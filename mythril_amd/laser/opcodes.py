"""Opcode names of the LASER opcode table (support/opcodes.py:16-144).

Byte values are the EVM's; the 146 names and their bytes are pinned against the
reference table by tests/test_laser_host.py (tests/golden/opcodes.json, emitted
from the reference's own opcodes.py).  Gas and required-stack counts are taken
from libmythgpu.so (mg_opcode_info) so the host and the device share one table.
"""
from __future__ import annotations

from typing import Dict

_NAMED = {
    0x00: "STOP", 0x01: "ADD", 0x02: "MUL", 0x03: "SUB", 0x04: "DIV", 0x05: "SDIV", 0x06: "MOD",
    0x07: "SMOD", 0x08: "ADDMOD", 0x09: "MULMOD", 0x0A: "EXP", 0x0B: "SIGNEXTEND",
    0x10: "LT", 0x11: "GT", 0x12: "SLT", 0x13: "SGT", 0x14: "EQ", 0x15: "ISZERO", 0x16: "AND",
    0x17: "OR", 0x18: "XOR", 0x19: "NOT", 0x1A: "BYTE", 0x1B: "SHL", 0x1C: "SHR", 0x1D: "SAR",
    0x20: "SHA3",
    0x30: "ADDRESS", 0x31: "BALANCE", 0x32: "ORIGIN", 0x33: "CALLER", 0x34: "CALLVALUE",
    0x35: "CALLDATALOAD", 0x36: "CALLDATASIZE", 0x37: "CALLDATACOPY", 0x38: "CODESIZE",
    0x39: "CODECOPY", 0x3A: "GASPRICE", 0x3B: "EXTCODESIZE", 0x3C: "EXTCODECOPY",
    0x3D: "RETURNDATASIZE", 0x3E: "RETURNDATACOPY", 0x3F: "EXTCODEHASH",
    0x40: "BLOCKHASH", 0x41: "COINBASE", 0x42: "TIMESTAMP", 0x43: "NUMBER", 0x44: "DIFFICULTY",
    0x45: "GASLIMIT", 0x46: "CHAINID", 0x47: "SELFBALANCE", 0x48: "BASEFEE",
    0x50: "POP", 0x51: "MLOAD", 0x52: "MSTORE", 0x53: "MSTORE8", 0x54: "SLOAD", 0x55: "SSTORE",
    0x56: "JUMP", 0x57: "JUMPI", 0x58: "PC", 0x59: "MSIZE", 0x5A: "GAS", 0x5B: "JUMPDEST",
    0x5C: "BEGINSUB", 0x5D: "RETURNSUB", 0x5E: "JUMPSUB",
    0xF0: "CREATE", 0xF1: "CALL", 0xF2: "CALLCODE", 0xF3: "RETURN", 0xF4: "DELEGATECALL",
    0xF5: "CREATE2", 0xFA: "STATICCALL", 0xFD: "REVERT", 0xFE: "INVALID", 0xFF: "SELFDESTRUCT",
}


def _table() -> Dict[int, str]:
    t = dict(_NAMED)
    for k in range(32):
        t[0x60 + k] = f"PUSH{k + 1}"
    for k in range(16):
        t[0x80 + k] = f"DUP{k + 1}"
        t[0x90 + k] = f"SWAP{k + 1}"
    for k in range(5):
        t[0xA0 + k] = f"LOG{k}"
    return t


ADDRESS_OPCODE_MAPPING: Dict[int, str] = _table()
OPCODES: Dict[str, int] = {name: b for b, name in ADDRESS_OPCODE_MAPPING.items()}


def push_width(name: str) -> int:
    return int(name[4:]) if name.startswith("PUSH") else 0


_INFO: Dict[str, tuple] = {}


def _info(op_code: str):
    if op_code not in _INFO:
        import ctypes
        from .. import native
        lib = native.load()
        gmin, gmax, req = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        rc = lib.mg_opcode_info(OPCODES[op_code], ctypes.byref(gmin), ctypes.byref(gmax),
                                ctypes.byref(req))
        _INFO[op_code] = (0, 0, 0) if rc != 0 else (gmin.value, gmax.value, req.value)
    return _INFO[op_code]


def get_required_stack_elements(op_code: str) -> int:
    """instruction_data.get_required_stack_elements (instruction_data.py:51-56), with
    the reference table's counts (ADDMOD 2, SSTORE 1, DUP/SWAP 0 ...)."""
    return _info(op_code)[2]


def get_opcode_gas(op_code: str):
    """instruction_data.get_opcode_gas (instruction_data.py:43-48)."""
    return _info(op_code)[:2]
