"""C3 on the MI355X (BASELINE configs[2]): the assembled BECToken
(tests/bectoken.py) -- its CVE-2018-10299 transaction on kernel 1 equal to the
oracle's, and ``myth analyze BECToken.sol -t 2`` with every module on kernels 1
and 2 and the exact procedure: SWC-101 at batchTransfer's multiplication, no
path dropped, nothing left unknown."""
import pytest

import bectoken

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.device import GpuDevice
    d = GpuDevice(0)
    yield d
    d.close()


def test_the_overflow_concretely_on_kernel1(dev):
    from oracle_device import OracleDevice
    assert bectoken.concrete_exploit(dev) == bectoken.concrete_exploit(OracleDevice())


def test_myth_analyze_bectoken_t2(dev, monkeypatch, tmp_path):
    import analyze
    from fnames import use_signature_db
    use_signature_db(monkeypatch, tmp_path)
    issues, info = analyze.analyze("BECToken", None, 2, dev, dev, code=bectoken.creation(), search=False)
    table = analyze.issue_table(issues)
    assert ("101", bectoken.mul_address(), "batchTransfer(address[],uint256)", "Integer Arithmetic Bugs") in table, table
    assert info["escapes_dropped"] == 0
    assert info["confirmations"]["unknown"] == 0 and info["fork_filter"]["unknown"] == 0
    assert info["cache"]["lru_hits"] + info["cache"]["seed_hits"] > 0 and info["exact"]["calls"] > 0
