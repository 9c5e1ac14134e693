"""KillBilly (solidity_examples/killbilly.sol) as EVM bytecode, assembled here --
TEST INFRASTRUCTURE, the C1 stand-in.

There is no solc in this image, so ``myth analyze killbilly.sol -t 3`` cannot
compile the source.  This module writes the contract the way solc 0.5 lays it
out -- a constructor that clears ``is_killable`` and returns the runtime code,
a dispatcher of PUSH4 <selector> EQ PUSH2 <entry> JUMPI rows (the pattern
Disassembly's function table reads), a call-value check per function,
``is_killable`` as the low byte of slot 0 and ``approved_killers[a]`` at
keccak256(pad32(a) . pad32(1)) -- and assembles it.  The selectors are
keccak256 of the text signatures, so the function names resolve through the
signature database like the compiled contract's.  Addresses differ from solc's
output (the README's PC 354 is solc's); the semantics are the source's:

* killerize(address addr):      approved_killers[addr] = true
* activatekillability():        require(approved_killers[msg.sender] == true); is_killable = true
* commencekilling():            require(is_killable); selfdestruct(msg.sender)
* is_killable(), approved_killers(address): the public getters.
"""
from __future__ import annotations

from typing import Dict, List, Tuple, Union

from mythril_amd.keccak import keccak256
from mythril_amd.laser.opcodes import OPCODES

SIGNATURES = ["is_killable()", "approved_killers(address)", "killerize(address)", "activatekillability()",
              "commencekilling()"]


def selector(sig: str) -> int:
    return int.from_bytes(keccak256(sig.encode())[:4], "big")


Item = Union[str, Tuple[str, object]]


def assemble(items: List[Item]) -> bytes:
    """items: an opcode name, ("PUSHn", int), ("PUSH2", "@label") or
    ("LABEL", name) (a JUMPDEST with that name).  Two passes: every PUSH of a
    label is PUSH2, so addresses are known after the first."""
    labels: Dict[str, int] = {}
    for final in (False, True):
        out = bytearray()
        for it in items:
            if isinstance(it, str):
                out.append(OPCODES[it])
            elif it[0] == "LABEL":
                labels[it[1]] = len(out)
                out.append(OPCODES["JUMPDEST"])
            else:
                name, arg = it
                n = int(name[4:])
                v = labels.get(arg[1:], 0) if isinstance(arg, str) else int(arg)
                if final and isinstance(arg, str) and arg[1:] not in labels:
                    raise KeyError(arg)
                out.append(OPCODES[name])
                out += v.to_bytes(n, "big")
    return bytes(out)


def _nonpayable(fn: str) -> List[Item]:
    """solc's per-function call-value check."""
    return [("LABEL", fn), "CALLVALUE", "DUP1", "ISZERO", ("PUSH2", f"@{fn}_ok"), "JUMPI",
            ("PUSH1", 0), "DUP1", "REVERT", ("LABEL", f"{fn}_ok"), "POP"]


def _mapping_slot_of_top() -> List[Item]:
    """keccak256(pad32(stack top) . pad32(1)): approved_killers' slot (consumes the key)."""
    return [("PUSH1", 0), "MSTORE", ("PUSH1", 1), ("PUSH1", 0x20), "MSTORE", ("PUSH1", 0x40), ("PUSH1", 0), "SHA3"]


def _address_arg() -> List[Item]:
    """abi.decode of one address argument (calldata long enough, else revert)."""
    return [("PUSH1", 0x24), "CALLDATASIZE", "LT", ("PUSH2", "@revert"), "JUMPI",
            ("PUSH1", 4), "CALLDATALOAD", ("PUSH20", (1 << 160) - 1), "AND"]


def _set_low_byte() -> List[Item]:
    """storage[slot] = (storage[slot] & ~0xff) | 1, slot on the stack (consumed)."""
    return ["DUP1", "SLOAD", ("PUSH1", 0xFF), "NOT", "AND", ("PUSH1", 1), "OR", "SWAP1", "SSTORE"]


def runtime() -> bytes:
    sel = {s: selector(s) for s in SIGNATURES}
    items: List[Item] = [("PUSH1", 0x80), ("PUSH1", 0x40), "MSTORE",
                         ("PUSH1", 4), "CALLDATASIZE", "LT", ("PUSH2", "@revert"), "JUMPI",
                         ("PUSH1", 0), "CALLDATALOAD", ("PUSH1", 0xE0), "SHR"]
    entries = {"is_killable()": "get_killable", "approved_killers(address)": "get_approved",
               "killerize(address)": "killerize", "activatekillability()": "activate",
               "commencekilling()": "commence"}
    for s in SIGNATURES:
        items += ["DUP1", ("PUSH4", sel[s]), "EQ", ("PUSH2", "@" + entries[s]), "JUMPI"]
    items += [("LABEL", "revert"), ("PUSH1", 0), "DUP1", "REVERT"]
    # is_killable(): return the low byte of slot 0 as a bool word
    items += _nonpayable("get_killable") + [
        ("PUSH1", 0), "SLOAD", ("PUSH1", 0xFF), "AND", "ISZERO", "ISZERO",
        ("PUSH1", 0x80), "MSTORE", ("PUSH1", 0x20), ("PUSH1", 0x80), "RETURN"]
    # approved_killers(address)
    items += _nonpayable("get_approved") + _address_arg() + _mapping_slot_of_top() + [
        "SLOAD", ("PUSH1", 0xFF), "AND", "ISZERO", "ISZERO",
        ("PUSH1", 0x80), "MSTORE", ("PUSH1", 0x20), ("PUSH1", 0x80), "RETURN"]
    # killerize(address addr): approved_killers[addr] = true
    items += _nonpayable("killerize") + _address_arg() + _mapping_slot_of_top() + _set_low_byte() + ["STOP"]
    # activatekillability(): require(approved_killers[msg.sender] == true); is_killable = true
    items += _nonpayable("activate") + ["CALLER"] + _mapping_slot_of_top() + [
        "SLOAD", ("PUSH1", 0xFF), "AND", ("PUSH1", 1), "EQ", "ISZERO", ("PUSH2", "@revert"), "JUMPI",
        ("PUSH1", 0)] + _set_low_byte() + ["STOP"]
    # commencekilling(): require(is_killable); selfdestruct(msg.sender)
    items += _nonpayable("commence") + [
        ("PUSH1", 0), "SLOAD", ("PUSH1", 0xFF), "AND", "ISZERO", ("PUSH2", "@revert"), "JUMPI",
        "CALLER", "SELFDESTRUCT"]
    return assemble(items)


def creation() -> bytes:
    """Constructor (non-payable; is_killable = false) + CODECOPY / RETURN of the
    runtime code appended after it."""
    rt = runtime()
    head: List[Item] = [("PUSH1", 0x80), ("PUSH1", 0x40), "MSTORE",
                        "CALLVALUE", "DUP1", "ISZERO", ("PUSH2", "@ok"), "JUMPI", ("PUSH1", 0), "DUP1", "REVERT",
                        ("LABEL", "ok"), "POP",
                        ("PUSH1", 0), "DUP1", "SLOAD", ("PUSH1", 0xFF), "NOT", "AND", "SWAP1", "SSTORE",
                        ("PUSH2", len(rt)), "DUP1", ("PUSH2", 0), ("PUSH1", 0), "CODECOPY", ("PUSH1", 0), "RETURN"]
    n = len(assemble(head))
    head[-5] = ("PUSH2", n)                  # the runtime code starts right after the head
    return assemble(head) + rt


def selfdestruct_address() -> int:
    """Byte address of the SELFDESTRUCT in the runtime code."""
    from mythril_amd.laser.disassembly import Disassembly
    d = Disassembly(runtime())
    return next(i["address"] for i in d.instruction_list if i["opcode"] == "SELFDESTRUCT")
