"""Contract creation through the LASER mirror (concolic.execute_contract_creation,
transaction_models.py:206-284): the reference's creation-code fixtures
(tests/testdata/inputs/*.sol.o with a constructor, tests/golden/bytecodes.json)
deployed from an attacker-like creator, then one message call into the
installed runtime code.  Shared by the CPU (oracle device) and GPU tests."""
import json
from pathlib import Path

from mythril_amd.laser import (Account, LaserEVM, WorldState, execute_contract_creation,
                               execute_message_call, generate_contract_address)

GOLDEN = Path(__file__).resolve().parent / "golden"
CREATOR = 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE     # transaction/symbolic.py:31 (CREATOR)
ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF
# creation codes among the fixtures (constructor prologue CALLVALUE / CODECOPY)
CREATION = ["exceptions_0.8.0.sol.o", "extcall.sol.o", "flag_array.sol.o",
            "symbolic_exec_bytecode.sol.o"]


def creation_code(name: str) -> bytes:
    return bytes.fromhex(json.loads((GOLDEN / "bytecodes.json").read_text())[name])


def deploy(dev, name: str, value: int = 0):
    """(laser_evm, final_states, address) after one concolic creation."""
    ws = WorldState()
    creator = Account(CREATOR, concrete_storage=True)
    creator.set_balance(10 ** 20)
    ws.put_account(creator)
    laser_evm = LaserEVM(requires_statespace=False, device=dev)
    laser_evm.open_states = [ws]
    address = generate_contract_address(CREATOR, 0)
    finals = execute_contract_creation(laser_evm, None, CREATOR, CREATOR, creation_code(name),
                                       gas_limit=8_000_000, gas_price=1, value=value, track_gas=True)
    return laser_evm, finals, address


def call(laser_evm, address: int, data: bytes, value: int = 0):
    return execute_message_call(laser_evm, callee_address=address, caller_address=ATTACKER,
                                origin_address=ATTACKER, data=data, gas_limit=8_000_000,
                                gas_price=1, value=value, track_gas=True)


def summary(laser_evm, address: int):
    """Per open world state: (installed code, storage, creator nonce) — what parity compares."""
    out = []
    for ws in laser_evm.open_states:
        acct = ws[address]
        code = acct.code.raw if hasattr(acct.code, "raw") else acct.code
        out.append((bytes(code), sorted(acct.storage.items()), ws[CREATOR].nonce))
    return out
