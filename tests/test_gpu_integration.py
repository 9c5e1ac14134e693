"""analysis_tests.py:9-54's issue-count rows on the MI355X: kernel 1 steps the
creation and message-call paths (concrete and symbolic lanes), kernel 2
answers the fork filters and the SAT-only issue confirmations (model cache,
witness seeds, guided search).  Same harness and assertions as
tests/test_integration_cpu.py (which runs them on the C oracles)."""
import pytest

from test_integration_cpu import GOLDEN, check_row

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.device import GpuDevice
    d = GpuDevice(0)
    yield d
    d.close()


@pytest.mark.parametrize("row", GOLDEN["issue_counts"], ids=lambda r: f"{r[0]}-{r[1]}")
def test_issue_counts_on_the_mi355x(row, dev):
    issues, info = check_row(row, dev, dev)
    assert info["lane_steps"] > 0            # kernel 1 stepped the paths
    assert info["kernel2_launches"] > 0      # kernel 2 answered the queries
