"""The reference's integration rows on the MI355X: kernel 1 steps the creation
and message-call paths (concrete and symbolic lanes), kernel 2 answers the fork
filters, the delayed strategy's quick-sat gate and the SAT-only issue
confirmations (model cache, witness seeds, guided search).  Same harness and
assertions as tests/test_integration_cpu.py (which runs them on the C oracles):
analysis_tests.py:9-82 (issue count, SWC id and function of every issue, BFS
and --strategy delayed), test_safe_functions.py:26-51 (0 / 2 / 4 safe
functions), the C1 stand-in (suicide.sol.o -t 3, default modules) and
KillBilly -t 3 (tests/killbilly.py)."""
import pytest

from fnames import use_signature_db
from test_integration_cpu import GOLDEN, check_c1, check_killbilly, check_row, check_safe_functions

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.device import GpuDevice
    d = GpuDevice(0)
    yield d
    d.close()


@pytest.mark.parametrize("strategy", ["bfs", "delayed"])
@pytest.mark.parametrize("row", GOLDEN["issue_counts"], ids=lambda r: f"{r[0]}-{r[1]}")
def test_issue_counts_on_the_mi355x(row, strategy, dev, monkeypatch, tmp_path):
    use_signature_db(monkeypatch, tmp_path)
    issues, info = check_row(row, dev, dev, strategy=strategy)
    assert info["lane_steps"] > 0            # kernel 1 stepped the paths
    assert info["kernel2_launches"] > 0      # kernel 2 answered the queries


@pytest.mark.parametrize("row", GOLDEN["safe_functions"], ids=lambda r: r[0])
def test_safe_functions_on_the_mi355x(row, dev, monkeypatch, tmp_path):
    use_signature_db(monkeypatch, tmp_path)
    got, issues, info = check_safe_functions(row, dev, dev)
    if row[0] != "ether_send.sol.o":
        assert got == sorted(row[1])
    assert info["lane_steps"] > 0


@pytest.mark.parametrize("runtime", [True, False], ids=["bin-runtime", "creation"])
def test_c1_stand_in_on_the_mi355x(runtime, dev, monkeypatch, tmp_path):
    use_signature_db(monkeypatch, tmp_path)
    check_c1(dev, dev, runtime)


def test_killbilly_on_the_mi355x(dev, monkeypatch, tmp_path):
    use_signature_db(monkeypatch, tmp_path)
    issues, info = check_killbilly(dev, dev)
    assert info["lane_steps"] > 0 and info["kernel2_launches"] > 0


@pytest.mark.parametrize("name", sorted(__import__("mythril_amd.workloads", fromlist=["x"]).bytecode_names()))
def test_all_modules_issue_set_equals_the_oracle_devices(name, dev, monkeypatch, tmp_path):
    """``myth analyze -f <code> -t 2`` with every module (bench.py's myth_analyze
    field): kernels 1 and 2 on the MI355X file the issue set the same harness
    files on the C oracles, where every symbolic instruction is the host
    restatement's (tests/symref.py) -- taint lanes, symbolic lanes and their
    escapes included."""
    import analyze
    from oracle_device import OracleDevice, OracleK2
    use_signature_db(monkeypatch, tmp_path)
    gi, ginfo = analyze.analyze(name, None, 2, dev, dev)
    ci, cinfo = analyze.analyze(name, None, 2, OracleDevice(), OracleK2())
    assert analyze.issue_table(gi) == analyze.issue_table(ci), (ginfo, cinfo)
    assert ginfo["escapes_dropped"] == cinfo["escapes_dropped"]
    # the run itself, not only its issues -- the fork events
    # (a JUMPI the device tagged symbolic whose term folds to a constant is no
    # fork), the fork filter's verdicts, every confirmation and what the
    # solver backend answered
    assert ginfo["forks"] == cinfo["forks"], (ginfo["forks"], cinfo["forks"])
    ff = ("groups", "queries", "kept", "pruned", "unknown")      # not "flushes": how the device batches them
    assert {k: ginfo["fork_filter"][k] for k in ff} == {k: cinfo["fork_filter"][k] for k in ff}, (
        ginfo["fork_filter"], cinfo["fork_filter"])
    assert ginfo["confirmations"] == cinfo["confirmations"], (ginfo["confirmations"], cinfo["confirmations"])
    keys = ("calls", "refuted", "seed", "search", "unknown")
    assert {k: ginfo["search"][k] for k in keys} == {k: cinfo["search"][k] for k in keys}, (
        ginfo["search"], cinfo["search"])
