"""The statespace graph on an MI355X: with
requires_statespace every state is stepped one instruction at a time on kernel 1
(k_lane_step / k_sym_step, one-lane batches) and the graph is built per step as
svm.py:549-637 builds it.  On each contract the graph run ends the call in the
batched core's outcomes, satisfies the graph invariants, and equals the graph
the same run builds on the C oracle device node for node and edge for edge."""
import pytest

import statespace_cases as sc
from mythril_amd.device import GpuDevice
from oracle_device import OracleDevice

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


@pytest.mark.parametrize("name", sc.CONTRACTS)
def test_graph_on_the_device_equals_the_oracle_devices(dev, name, monkeypatch):
    got, laser = sc.run(dev, name, True, monkeypatch)
    plain, _ = sc.run(dev, name, False, monkeypatch)
    assert got == plain
    sc.check_graph(laser)
    _, ref = sc.run(OracleDevice(), name, True, monkeypatch)
    assert sc.shape(laser) == sc.shape(ref)


def test_branch_program_graph_on_the_device(dev, monkeypatch):
    _, laser = sc.run(dev, "Branch", True, monkeypatch, code=sc.BRANCH, signals=True)
    assert sorted(p for _, _, p, _ in sc.shape(laser)[0]) == sorted(tuple(v) for v in sc.BRANCH_PCS.values())
    _, ref = sc.run(OracleDevice(), "Branch", True, monkeypatch, code=sc.BRANCH, signals=True)
    assert sc.shape(laser) == sc.shape(ref)


@pytest.mark.parametrize("row", __import__("test_integration_cpu").GOLDEN["issue_counts"],
                         ids=lambda r: f"{r[0]}-{r[1]}")
def test_analysis_rows_with_the_graph_on_the_device(dev, row, monkeypatch, tmp_path):
    """analysis_tests.py's rows with requires_statespace on kernels 1 and 2:
    the reference's counts, SWC ids and functions (flag_array's calldata too).
    symbolic_exec_bytecode's constructor copies its arguments into a full
    arena: the single step regrows the lane and runs it in the grown batch
    (a regrown lane is not a stepped successor)."""
    import test_integration_cpu as ti
    from fnames import use_signature_db
    use_signature_db(monkeypatch, tmp_path)
    ti.check_row(row, dev, dev, statespace=True)
