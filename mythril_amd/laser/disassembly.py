"""Host disassembly: the instruction list LASER indexes by pc, and the
dispatcher's function table.

Restates ``asm.disassemble`` (disassembler/asm.py:99-148) and ``Disassembly``
(disassembler/disassembly.py:9-114): the instruction list with pc = index, a
trailing bzzr swarm hash ignored when "bzzr" occurs in Python's ``str`` of the
last 43 bytes, unknown bytes as ``INVALID``, PUSH arguments as ``0x``-hex
(truncated at the end of code); ``get_easm``; and the function table built from
the ``PUSH1..PUSH4 EQ PUSHn`` dispatcher pattern (``func_hashes``,
``function_name_to_address``, ``address_to_function_name``, names from the
signature database or ``_function_0x<hash>``).  The device builds the same
instruction list and the same function-entry set in ``mg_load_code``; the three
(host, device, oracle) are compared in the tests.  ``LaserEVM`` switches
``environment.active_function_name`` from this table at every JUMP / JUMPI
successor (svm.py:549-637), which is what every detection module files its
issues under.
"""
from __future__ import annotations

import os
import sqlite3
from collections import defaultdict
from typing import DefaultDict, Dict, Iterator, List, Optional, Tuple, Union

from .opcodes import ADDRESS_OPCODE_MAPPING, OPCODES, push_width


def _decode(code: Union[str, bytes, bytearray]) -> bytes:
    """ethereum/util.py safe_decode for text; bytes as given."""
    if isinstance(code, str):
        return bytes.fromhex(code[2:] if code.startswith("0x") else code)
    return bytes(code)


def disassemble(bytecode: Union[str, bytes, bytearray]) -> List[Dict]:
    """asm.disassemble: list of {"address", "opcode"[, "argument"]}."""
    bytecode = _decode(bytecode)
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


def instruction_list_to_easm(instruction_list: List[Dict]) -> str:
    """asm.py:38-52: one "<address> <opcode>[ <argument>]" line per instruction."""
    lines = []
    for ins in instruction_list:
        lines.append(f"{ins['address']} {ins['opcode']}" + (f" {ins['argument']}" if "argument" in ins else "") + "\n")
    return "".join(lines)


def get_opcode_from_name(operation_name: str) -> int:
    """asm.py:55-63."""
    if operation_name in OPCODES:
        return OPCODES[operation_name]
    raise RuntimeError("Unknown opcode")


def is_sequence_match(pattern: List, instruction_list: List[Dict], index: int) -> bool:
    """asm.py:79-93: instruction index + k has an opcode in pattern[k] for every k."""
    if index + len(pattern) > len(instruction_list):
        return False
    return all(instruction_list[index + k]["opcode"] in slot for k, slot in enumerate(pattern))


def find_op_code_sequence(pattern: List, instruction_list: List[Dict]) -> Iterator[int]:
    """asm.py:66-76: every index where the pattern starts."""
    for i in range(0, len(instruction_list) - len(pattern) + 1):
        if is_sequence_match(pattern, instruction_list, i):
            yield i


# ------------------------------------------------------------------ signatures
class SignatureDB:
    """The local part of support/signatures.py:117-235: a byte signature ->
    text signatures lookup in ``$MYTHRIL_DIR/signatures.db`` (else
    ``~/.mythril/signatures.db``; the same sqlite schema: table ``signatures``
    (byte_sig, text_sig)), plus the signatures of Solidity files added this run.
    Online lookup (4byte.directory) is not available: there is no network.  A
    missing database file is read as empty and not created."""

    _instances: Dict[str, "SignatureDB"] = {}

    def __new__(cls, enable_online_lookup: bool = False, path: Optional[str] = None):
        # support/signatures.py:45-63: one instance per process (Singleton)
        base = path or os.environ.get("MYTHRIL_DIR") or os.path.join(os.path.expanduser("~"), ".mythril")
        key = os.path.join(base, "signatures.db")
        inst = cls._instances.get(key)
        if inst is None:
            inst = super().__new__(cls)
            inst.path = key
            inst.enable_online_lookup = enable_online_lookup
            inst.solidity_sigs: DefaultDict[str, List[str]] = defaultdict(list)
            cls._instances[key] = inst
        return inst

    @staticmethod
    def _normalize_byte_sig(byte_sig: str) -> str:
        if not byte_sig.startswith("0x"):
            byte_sig = "0x" + byte_sig
        if len(byte_sig) != 10:
            raise ValueError("Invalid byte signature %s, must have 10 characters" % byte_sig)
        return byte_sig

    def add(self, byte_sig: str, text_sig: str) -> None:
        byte_sig = self._normalize_byte_sig(byte_sig)
        os.makedirs(os.path.dirname(self.path), exist_ok=True)
        with sqlite3.connect(self.path) as conn:
            conn.execute("CREATE TABLE IF NOT EXISTS signatures(byte_sig VARCHAR(10), text_sig VARCHAR(255),"
                         "PRIMARY KEY (byte_sig, text_sig))")
            conn.execute("INSERT OR IGNORE INTO signatures (byte_sig, text_sig) VALUES (?,?)",
                         (byte_sig, text_sig))

    def get(self, byte_sig: str, online_timeout: int = 2) -> List[str]:
        """signatures.py:183-225 without the online step: the Solidity signatures
        of this run, else the local database's rows."""
        byte_sig = self._normalize_byte_sig(byte_sig)
        text_sigs = self.solidity_sigs.get(byte_sig)
        if text_sigs is not None:
            return text_sigs
        if not os.path.isfile(self.path):
            return []
        with sqlite3.connect(self.path) as conn:
            try:
                rows = conn.execute("SELECT text_sig FROM signatures WHERE byte_sig=?", (byte_sig,)).fetchall()
            except sqlite3.OperationalError:          # no table yet
                return []
        return [r[0] for r in rows]

    def __getitem__(self, item: str) -> List[str]:
        return self.get(byte_sig=item)

    def add_sigs(self, file_path: str, solc_json) -> None:
        """signatures.py:239-250: solc's methodIdentifiers of every contract."""
        for contract in solc_json["contracts"][file_path].values():
            if "methodIdentifiers" not in contract["evm"]:
                continue
            for name, hash_ in contract["evm"]["methodIdentifiers"].items():
                sig = "0x{}".format(hash_)
                self.solidity_sigs[sig].append(name)
                self.add(sig, name)

    @classmethod
    def _reset(cls) -> None:
        """Forget every instance (tests point MYTHRIL_DIR elsewhere)."""
        cls._instances.clear()


def get_function_info(index: int, instruction_list: List[Dict],
                      signature_database: SignatureDB) -> Tuple[str, Optional[int], Optional[str]]:
    """disassembly.py:64-114: (function hash, entry point, function name) of the
    dispatcher entry whose PUSH is at ``index``."""
    function_hash = "0x" + instruction_list[index]["argument"][2:].rjust(8, "0")
    function_names = signature_database.get(function_hash)
    if len(function_names) > 0:
        # the reference joins a set: its order is Python's, for one name it is the name
        function_name = " or ".join(set(function_names))
    else:
        function_name = "_function_" + function_hash
    try:
        offset = instruction_list[index + 2]["argument"]
    except (KeyError, IndexError):
        return function_hash, None, None
    if offset == "0x":
        # int("0x", 16) raises in the reference (a PUSH cut off by the end of
        # the code); no entry point here
        return function_hash, None, None
    return function_hash, int(offset, 16), function_name


class Disassembly:
    """Disassembly(code): ``bytecode`` (as given), ``instruction_list`` and the
    dispatcher's function table."""

    def __init__(self, code: Union[str, bytes, bytearray], enable_online_lookup: bool = False):
        self.bytecode = code
        self.raw = _decode(code)
        self.instruction_list = disassemble(self.raw)
        self.func_hashes: List[str] = []
        self.function_name_to_address: Dict[str, int] = {}
        self.address_to_function_name: Dict[int, str] = {}
        self.enable_online_lookup = enable_online_lookup
        self.assign_bytecode(bytecode=code)

    def assign_bytecode(self, bytecode) -> None:
        """disassembly.py:36-54."""
        self.bytecode = bytecode
        signatures = SignatureDB(enable_online_lookup=self.enable_online_lookup)
        self.instruction_list = disassemble(bytecode)
        jump_table_indices = find_op_code_sequence([("PUSH1", "PUSH2", "PUSH3", "PUSH4"), ("EQ",)],
                                                   self.instruction_list)
        for index in jump_table_indices:
            function_hash, jump_target, function_name = get_function_info(index, self.instruction_list,
                                                                          signatures)
            self.func_hashes.append(function_hash)
            if jump_target is not None and function_name is not None:
                self.function_name_to_address[function_name] = jump_target
                self.address_to_function_name[jump_target] = function_name
        self._entry_names = None

    def get_easm(self) -> str:
        return instruction_list_to_easm(self.instruction_list)

    def __len__(self):
        return len(self.instruction_list)

    # ---- the batched core's view of the table -------------------------------
    def function_entries(self) -> List[int]:
        """uint8 per instruction index: 1 where a JUMP / JUMPI landing switches
        active_function_name (its address is a key of address_to_function_name,
        or it is address 0) -- what mg_load_code computes on the device."""
        out = [0] * len(self.instruction_list)
        for k, ins in enumerate(self.instruction_list):
            if ins["address"] in self.address_to_function_name or ins["address"] == 0:
                out[k] = 1
        return out

    def name_at(self, index: int) -> Optional[str]:
        """_new_node_state's switch (svm.py:617-633) for a successor at
        instruction ``index``: the entry's name, "fallback" at address 0, or
        None (the name stays)."""
        try:
            address = self.instruction_list[index]["address"]
        except IndexError:
            return None
        name = self.address_to_function_name.get(address)
        if name is not None:
            return name
        return "fallback" if address == 0 else None
