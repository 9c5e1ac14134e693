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
