"""The host LASER mirror end to end on CPU: the reference's VMTests harness
(evm_test.py:124-189) through LaserEVM + execute_message_call, stepping on the
oracle-backed device (tests/oracle_device.py) instead of kernel 1.  The same
harness runs on kernel 1 in test_gpu_laser.py; together they pin the host layer
and the device to the reference's expected post-states."""
import test_gpu_laser as tg
from oracle_device import OracleDevice
from vmtests_util import load_vmtests


def test_vmtests_through_laser_evm_on_the_oracle_device():
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    escaping = tg._oracle_escapes(vectors)      # before the device: one oracle registry
    dev = OracleDevice()
    passed = 0
    for v in vectors:
        if v["name"] in escaping:
            continue
        laser_evm, final_states = tg._run_vmtest(dev, v)
        gas_used = v["gas_used"]
        if gas_used is not None and gas_used < int(v["block_gas_limit"]):
            assert any(s.mstate.min_gas_used <= gas_used for s in final_states), v["name"]
        if v["post"] == {}:
            assert len(laser_evm.open_states) == 0, v["name"]
        else:
            assert len(laser_evm.open_states) == 1, v["name"]
            ws = laser_evm.open_states[0]
            for address, details in v["post"].items():
                acct = ws[int(address, 16)]
                for index, value in details["storage"].items():
                    assert acct.storage[int(index, 16)].value == int(value, 16), v["name"]
        passed += 1
    assert passed == 499
