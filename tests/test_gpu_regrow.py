"""Capacity escapes resumed inside their batch on an MI355X (kernel 1 +
mg_lanes_alloc re-allocation): the event log equals a run with large
capacities from the start (tests/test_regrow_cpu.py on the oracle device)."""
import pytest

from mythril_amd.device import GpuDevice
from mythril_amd.laser import BreadthFirstSearchStrategy, DepthFirstSearchStrategy
from test_regrow_cpu import _run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


@pytest.mark.parametrize("strategy", [BreadthFirstSearchStrategy, DepthFirstSearchStrategy])
def test_regrown_lanes_keep_the_event_order_on_the_gpu(dev, strategy):
    log_big, open_big, regrows_big, steps_big = _run(strategy, 64, dev)
    log, opened, regrows, steps = _run(strategy, 1, dev)
    assert regrows_big == 0 and regrows >= 2
    assert steps == steps_big
    assert log == log_big
    assert opened == open_big
    # and the oracle device agrees with both
    log_o, open_o, _, steps_o = _run(strategy, 1)
    assert (log_o, open_o, steps_o) == (log, opened, steps)
