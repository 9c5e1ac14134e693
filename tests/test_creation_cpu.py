"""Contract creation on the oracle device (CPU): address derivation, runtime-code
installation, constructor value checks, argument constructors escaping, and a
message call into the deployed code."""
from creation_util import call, creation_code, deploy, summary
from oracle_device import OracleDevice

from mythril_amd.laser import generate_contract_address


def test_contract_address_known_answers():
    # keccak256(rlp([sender, nonce]))[12:] for a widely published sender
    s = 0x6AC7EA33F8831EA9DCC53393AAA88B25A785DBF0
    assert generate_contract_address(s, 0) == 0xCD234A471B72BA2F1CCF0A70FCABA648A5EECD8D
    assert generate_contract_address(s, 1) == 0x343C43A37D37DFF08AE8C4A11544C718ABB4FCF8
    assert generate_contract_address(s, 2) == 0xF778B86FA74E846C4F0A1FBD1335FE81C00A0C91
    assert generate_contract_address(s, 3) == 0xFFFD933A0BC612844EAF0C6FE3E5B8E9B6C1D19C



def test_contract_address_leading_zero_creator():
    """The reference passes the creator as an int (world_state.py:171,237), so rlp
    writes it like any integer: minimal big-endian bytes.  A creator whose top
    byte is 0 is therefore shorter than 20 bytes in the preimage (here 2 bytes:
    0x82 0x12 0x34), then the nonce (0 -> 0x80), under a 0xc4 list header."""
    from mythril_amd.keccak import keccak256
    want = int.from_bytes(keccak256(bytes([0xC4, 0x82, 0x12, 0x34, 0x80]))[12:], "big")
    assert generate_contract_address(0x1234, 0) == want
    want1 = int.from_bytes(keccak256(bytes([0xC4, 0x82, 0x12, 0x34, 0x01]))[12:], "big")
    assert generate_contract_address(0x1234, 1) == want1


def _installed(name, value=0):
    laser_evm, finals, addr = deploy(OracleDevice(), name, value)
    return laser_evm, finals, addr


def test_argumentless_constructors_install_runtime_code():
    for name in ("exceptions_0.8.0.sol.o",):
        laser_evm, _, addr = _installed(name)
        (code, storage, nonce), = summary(laser_evm, addr)
        assert code and code in creation_code(name), name      # runtime code is embedded
        assert nonce == 1, name                                 # creator nonce bumped
        ws = laser_evm.open_states[0]
        assert ws[addr].code.instruction_list, name


def test_constructor_value_check():
    # flag_array's constructor requires msg.value == 0.1 ether (require in the ctor)
    laser_evm, _, _ = _installed("flag_array.sol.o", value=0)
    assert laser_evm.open_states == []
    laser_evm, _, addr = _installed("flag_array.sol.o", value=10 ** 17)
    assert len(laser_evm.open_states) == 1
    ws = laser_evm.open_states[0]
    assert ws[addr].balance().value == 10 ** 17


def test_constructor_calling_out_escapes():
    # extcall's constructor CALLs another account: calls between contracts stay
    # on the host (out of scope here) -> without an escape handler the path ends
    laser_evm, _, _ = _installed("extcall.sol.o")
    assert laser_evm.open_states == []


def test_constructor_with_arguments_escapes():
    # reads its arguments past the code (CODESIZE / CODECOPY of symbolic calldata):
    # no escape handler -> the path is dropped, as the reference drops
    # NotImplementedError paths (svm.py:314-316)
    laser_evm, _, _ = _installed("symbolic_exec_bytecode.sol.o")
    assert laser_evm.open_states == []


def test_message_call_into_deployed_code():
    laser_evm, _, addr = _installed("exceptions_0.8.0.sol.o")
    code = laser_evm.open_states[0][addr].code
    names = [ins["opcode"] for ins in code.instruction_list]
    assert names[:3] == ["PUSH1", "PUSH1", "MSTORE"]          # a solc runtime prologue
    finals = call(laser_evm, addr, bytes(4))       # unknown selector -> revert, no open state
    assert finals and all(s.environment.code is not None for s in finals)
