"""Host disassembly: the instruction list LASER indexes by pc.

Restates ``asm.disassemble`` (disassembler/asm.py:99-148) and the parts of
``Disassembly`` (disassembler/disassembly.py:9-56) the execution loop uses: the
instruction list with pc = index, a trailing bzzr swarm hash ignored when
"bzzr" occurs in Python's ``str`` of the last 43 bytes, unknown bytes as
``INVALID``, PUSH arguments as ``0x``-hex (truncated at the end of code).  The
device builds the same list in ``mg_load_code``; the two are compared
instruction by instruction in tests/test_laser_host.py.  This is host metadata
for hooks (``get_current_instruction``), not a stepping path.
"""
from __future__ import annotations

from typing import Dict, List, Union

from .opcodes import ADDRESS_OPCODE_MAPPING, push_width


def _decode(code: Union[str, bytes, bytearray]) -> bytes:
    if isinstance(code, str):
        return bytes.fromhex(code[2:] if code.startswith("0x") else code)
    return bytes(code)


def disassemble(bytecode: bytes) -> List[Dict]:
    """asm.disassemble: list of {"address", "opcode"[, "argument"]}."""
    length = len(bytecode)
    if "bzzr" in str(bytes(bytecode[-43:])):
        length -= 43
    out: List[Dict] = []
    address = 0
    while address < length:
        name = ADDRESS_OPCODE_MAPPING.get(bytecode[address])
        if name is None:
            out.append({"address": address, "opcode": "INVALID"})
            address += 1
            continue
        ins = {"address": address, "opcode": name}
        w = push_width(name)
        if w:
            ins["argument"] = "0x" + bytecode[address + 1: address + 1 + w].hex()
            address += w
        out.append(ins)
        address += 1
    return out


class Disassembly:
    """Disassembly(code): ``bytecode`` (as given) and ``instruction_list``."""

    def __init__(self, code: Union[str, bytes, bytearray], enable_online_lookup: bool = False):
        self.bytecode = code
        self.raw = _decode(code)
        self.instruction_list = disassemble(self.raw)
        self.func_hashes: List[str] = []
        self.function_name_to_address: Dict[str, int] = {}
        self.address_to_function_name: Dict[int, str] = {}

    def __len__(self):
        return len(self.instruction_list)
