"""The reference's integration expectations (tests/integration_tests/
analysis_tests.py:9-54, as data in tests/golden/integration.json).

* SWC-115 row: TxOrigin's hooks (dependence_on_origin.py, restated in
  tests/refmodules.py) on concrete calls into origin.sol.o, batch-safe hooks as
  device actions.
* The four issue-count rows: ``myth analyze -f <code> -t 1 -m <module>
  --no-onchain-data`` on the batched core (tests/analyze.py): a symbolic
  creation and one symbolic message call through LaserEVM, escapes on the CPU
  restatement of the reference's mutators (tests/symref.py), the module
  restated (tests/refmodules.py), and issue confirmation SAT-only
  (mythril_amd.smt.search: kernel 2 over the model cache, the witness seeds and
  a guided search -- a model or "unknown", never "unsat").  Each row asserts
  the reference's issue count; an unconfirmed issue would be reported as
  "unknown", and the flag_array row also checks the reference's transaction
  input (analysis_tests.py:17).  Here the device is the C oracle (kernel 1) and
  oracle/bv_ref.c (kernel 2); tests/test_gpu_integration.py runs the same rows
  on the MI355X."""
import json
from pathlib import Path

import pytest

from mythril_amd.laser import BreadthFirstSearchStrategy

GOLDEN = json.loads((Path(__file__).resolve().parent / "golden" / "integration.json").read_text())


def test_origin_contract_reports_swc_115(monkeypatch):
    from test_taint_cpu import _run
    name, swc = GOLDEN["origin_swc"]
    assert name == "origin.sol.o"
    _, issues, _, _ = _run(BreadthFirstSearchStrategy, "device", monkeypatch, modules=("TxOrigin",))
    assert swc in {i[0] for i in issues}


def check_row(row, device, k2):
    """Run one analysis_tests.py row and assert the reference's outcome."""
    import analyze
    import refmodules
    name, module, tx_count, expected = row
    captured = {}
    cls = getattr(refmodules, module)
    orig_init = cls.__init__

    def init(self):
        orig_init(self)
        captured["module"] = self
    cls.__init__ = init
    try:
        issues, info = analyze.analyze(name, module, tx_count, device, k2)
    finally:
        cls.__init__ = orig_init
    assert info["escapes_dropped"] == 0, info
    assert len(issues) == expected, (name, module, [i[:3] for i in issues], info)
    if name == "flag_array.sol.o":
        # analysis_tests.py:11-17: the issue's test case, transaction 1 (0-based)
        steps = captured["module"].sequences[0]["steps"]
        assert steps[1]["input"] == GOLDEN_CALLDATA
    return issues, info


# analysis_tests.py:17 (the one exact calldata the reference's tests pin)
GOLDEN_CALLDATA = "0xab12585800000000000000000000000000000000000000000000000000000000000004d2"


@pytest.mark.parametrize("row", GOLDEN["issue_counts"], ids=lambda r: f"{r[0]}-{r[1]}")
def test_issue_counts_on_the_oracle_device(row):
    from oracle_device import OracleDevice, OracleK2
    check_row(row, OracleDevice(), OracleK2())
