"""The reference's integration expectations (tests/integration_tests/
analysis_tests.py:9-54, as data in tests/golden/integration.json).

The SWC-115 row runs here: TxOrigin's hooks (dependence_on_origin.py, restated
in tests/refmodules.py) on concrete calls into origin.sol.o, with the
batch-safe hooks as device actions (the C oracle stands in for kernel 1).  The
issue-count rows need the reference's full analysis -- symbolic transactions
whose issues are confirmed by an SMT backend (solver.get_transaction_sequence)
and the module set of `myth analyze` -- which this image lacks (no z3): they
are reported as skipped with that reason rather than silently absent."""
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


@pytest.mark.parametrize("row", GOLDEN["issue_counts"], ids=lambda r: f"{r[0]}-{r[1]}")
def test_issue_counts_blocked(row):
    name, module, tx_count, expected = row
    pytest.skip(f"blocked: {module} on {name} (-t {tx_count}, {expected} issue(s)) needs the reference's "
                "SMT-confirmed issue pipeline (solver.get_transaction_sequence); no SMT backend in this image")
