"""The reference's state tests as lane programs on kernel 1 (tests/state_pins.py):
the same expectations the CPU suite checks on the C oracle."""
import pytest

import state_pins
from mythril_amd.device import GpuDevice

pytestmark = pytest.mark.gpu


def test_lane_programs_on_the_device():
    dev = GpuDevice(0)
    try:
        state_pins.check(state_pins.run_programs(dev))
    finally:
        dev.close()


@pytest.mark.parametrize("name,code", state_pins.symbolic_programs())
def test_symbolic_fixture_programs_on_the_device(name, code):
    """The fixture's symbolic cases on k_sym_step, decoded and checked against
    the reference tests' verdicts and node for node against the restatement."""
    from copy import copy
    import symref
    from mythril_amd.lanes import LaneBatch
    from mythril_amd.laser import BreadthFirstSearchStrategy, LaserEVM
    dev = GpuDevice(0)
    try:
        vm = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy)
        s0 = state_pins.symbolic_state(code)
        shape = vm._shape([s0])
        b = LaneBatch(shape)
        vm._pack(b, 0, s0)
        b.steps[0] = 0
        dev.alloc(shape)
        dev.upload(b)
        dev.step()
        dev.download(b)
        assert int(b.status[0]) == 1, (name, int(b.status[0]), int(b.aux[0]))     # STOP on the device
        got = vm._materialise(b, 0, copy(s0))
        ref, eng = s0, symref.Engine()
        for _ in range(int(b.steps[0]) - 1):
            ref = eng.step(ref)[0]
        assert [x.raw for x in got.mstate.stack] == [x.raw for x in ref.mstate.stack]
        state_pins.check_symbolic_stack(name, got.mstate.stack)
    finally:
        dev.close()
