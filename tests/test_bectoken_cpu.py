"""tests/bectoken.py -- the assembled BECToken (C3) -- on the oracle device:
the dispatcher table names the source's functions, the constructor's storage
is the source's (owner, decimals, totalSupply = 7e9 * 10**18, the creator's
balance), and CVE-2018-10299 happens concretely: cnt * _value wraps to 0 and
two receivers are credited 2**255 by an account that holds nothing."""
import bectoken
from creation_util import ATTACKER, CREATOR
from mythril_amd.laser.disassembly import Disassembly


def test_dispatcher_names_the_source_functions(monkeypatch, tmp_path):
    from fnames import use_signature_db
    use_signature_db(monkeypatch, tmp_path)
    d = Disassembly(bectoken.runtime())
    assert sorted(d.address_to_function_name.values()) == sorted(bectoken.SIGNATURES)
    il = d.instruction_list
    assert next(i for i in il if i["address"] == bectoken.mul_address())["opcode"] == "MUL"


def test_the_overflow_concretely_on_the_oracle_device():
    from oracle_device import OracleDevice
    store = dict(bectoken.concrete_exploit(OracleDevice()))
    total = 7_000_000_000 * 10 ** 18
    assert store[0] == total                                        # totalSupply
    assert store[bectoken.balance_slot(CREATOR)] == total           # the creator keeps everything
    assert store[bectoken.balance_slot(0xA11CE)] == 1 << 255        # minted from nothing
    assert store[bectoken.balance_slot(0xB0B)] == 1 << 255
    assert store.get(bectoken.balance_slot(ATTACKER), 0) == 0       # amount wrapped to 0
    assert store[3] & ((1 << 160) - 1) == CREATOR and store[7] & 0xFF == 18
