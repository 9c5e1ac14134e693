"""Contract creation (concolic.execute_contract_creation) on kernel 1 vs the oracle
device: same open states, installed runtime code, storage, creator nonce and
final-state gas for every creation-code fixture and constructor value; then one
message call per selector into each deployed contract, compared the same way."""
import pytest

from creation_util import CREATION, call, deploy, summary
from mythril_amd.device import GpuDevice
from oracle_device import OracleDevice

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


def _gas(finals):
    return sorted((s.mstate.min_gas_used, s.mstate.max_gas_used) for s in finals or [])


@pytest.mark.parametrize("name", CREATION)
@pytest.mark.parametrize("value", [0, 10 ** 17])
def test_creation_device_equals_oracle(dev, name, value):
    g_evm, g_fin, addr = deploy(dev, name, value)
    o_evm, o_fin, _ = deploy(OracleDevice(), name, value)
    assert summary(g_evm, addr) == summary(o_evm, addr)
    assert _gas(g_fin) == _gas(o_fin)
    if not g_evm.open_states:
        return
    code = g_evm.open_states[0][addr].code
    selectors = sorted({int(ins["argument"], 16) for ins in code.instruction_list
                        if ins["opcode"] == "PUSH4"} | {0})[:8]
    for sel in selectors:                 # each call from a fresh deployment
        data = sel.to_bytes(4, "big") + bytes(64)
        g_evm, _, _ = deploy(dev, name, value)
        o_evm, _, _ = deploy(OracleDevice(), name, value)
        g_c = call(g_evm, addr, data)
        o_c = call(o_evm, addr, data)
        assert _gas(g_c) == _gas(o_c), hex(sel)
        assert summary(g_evm, addr) == summary(o_evm, addr), hex(sel)
