"""The reference's integration expectations on the batched core (CPU: the C
oracle as kernel 1, oracle/bv_ref.c as kernel 2; tests/test_gpu_integration.py
runs the same rows on the MI355X).

* SWC-115 row: TxOrigin's hooks on concrete calls into origin.sol.o, batch-safe
  hooks as device actions.
* analysis_tests.py:9-54 (``test_analysis``) and :71-82
  (``test_analysis_delayed``, ``--strategy delayed``): ``myth analyze -f <code>
  -t 1 -m <module>`` (tests/analyze.py).  Each row asserts the reference's issue
  count and, beyond it, every issue's SWC id and function: the function follows
  from the contract's source (tests/testdata/input_contracts), the dispatcher
  table and active_function_name (parity unpinned: the reference's tests assert
  counts only).  The flag_array row also checks the reference's transaction
  input (analysis_tests.py:17).  A confirmation that stays "unknown" is
  reported.
* test_safe_functions.py:26-51 (bytecode rows): ``myth safe-functions
  --bin-runtime -f <code>`` -- one transaction, all fourteen modules -- leaves
  0 / 2 / 4 safe functions in suicide / overflow / ether_send.
* The C1 stand-in: suicide.sol.o -t 3 with the default modules,
  deployed (--bin-runtime, the deployed ``kill(address)``) and as ``-f``
  creation code (the reference runs the runtime code as its constructor: the
  issue's function is ``constructor``).
* The README's C1 case itself, ``myth analyze killbilly.sol -t 3``: there is no
  solc here, so tests/killbilly.py assembles the contract from its source; the
  one issue is SWC-106 in commencekilling(), reached by killerize(attacker),
  activatekillability(), commencekilling() from the attacker -- the mapping
  slot keccak(addr . 1) written in transaction 1 must be the slot
  keccak(msg.sender . 1) read in transaction 2.

Function names come from a signature database holding the input contracts'
text signatures (tests/golden/signatures.json), as the reference's
~/.mythril/signatures.db does after importing them."""
import json
from pathlib import Path

import pytest

from fnames import use_signature_db
from mythril_amd.laser import BreadthFirstSearchStrategy

GOLDEN = json.loads((Path(__file__).resolve().parent / "golden" / "integration.json").read_text())

# analysis_tests.py:17 (the one exact calldata the reference's tests pin)
GOLDEN_CALLDATA = "0xab12585800000000000000000000000000000000000000000000000000000000000004d2"

# The issue set each row's count stands for: (SWC id, function), read off the
# contract's source (the reference's tests assert only the count).
EXPECTED = {
    ("flag_array.sol.o", "EtherThief"): [("105", "extractMoney(uint256)")],
    ("exceptions_0.8.0.sol.o", "Exceptions"): [("110", "assert1()"), ("110", "fail()")],
    ("symbolic_exec_bytecode.sol.o", "AccidentallyKillable"): [("106", "commencekilling()")],
    ("extcall.sol.o", "Exceptions"): [("110", "constructor")],
}


def test_origin_contract_reports_swc_115(monkeypatch):
    from test_taint_cpu import _run
    name, swc = GOLDEN["origin_swc"]
    assert name == "origin.sol.o"
    _, issues, _, _ = _run(BreadthFirstSearchStrategy, "device", monkeypatch, modules=("TxOrigin",))
    assert swc in {i[0] for i in issues}


def check_row(row, device, k2, strategy="bfs", statespace=False):
    """Run one analysis_tests.py row and assert the reference's outcome."""
    import analyze
    name, module, tx_count, expected = row
    issues, info = analyze.analyze(name, module, tx_count, device, k2, strategy=strategy,
                                   statespace=statespace)
    report = analyze.issue_table(issues)
    assert info["escapes_dropped"] == 0, info
    assert len(issues) == expected, (name, module, report, info)
    assert sorted((i.swc_id, i.function) for i in issues) == EXPECTED[(name, module)], (report, info)
    assert all(i.contract == "MAIN" for i in issues)
    if name == "flag_array.sol.o":
        # analysis_tests.py:11-17: the issue's test case, transaction 1 (0-based)
        assert issues[0].transaction_sequence["steps"][1]["input"] == GOLDEN_CALLDATA
    return issues, info


@pytest.mark.parametrize("row", GOLDEN["issue_counts"], ids=lambda r: f"{r[0]}-{r[1]}")
def test_issue_counts_on_the_oracle_device(row, monkeypatch, tmp_path):
    from oracle_device import OracleDevice, OracleK2
    use_signature_db(monkeypatch, tmp_path)
    check_row(row, OracleDevice(), OracleK2())


@pytest.mark.parametrize("row", GOLDEN["issue_counts"], ids=lambda r: f"{r[0]}-{r[1]}")
def test_issue_counts_delayed_strategy_on_the_oracle_device(row, monkeypatch, tmp_path):
    """analysis_tests.py:71-82: the same rows under --strategy delayed
    (DelayConstraintStrategy, constraint_strategy.py:19-47: kernel-2 quick-sat
    gates every state, the parked ones get a model from the backend)."""
    from oracle_device import OracleDevice, OracleK2
    assert GOLDEN["delayed"]
    use_signature_db(monkeypatch, tmp_path)
    check_row(row, OracleDevice(), OracleK2(), strategy="delayed")


def check_safe_functions(row, device, k2):
    import analyze
    name, safe = row
    got, issues, info = analyze.safe_functions(name, device, k2)
    assert info["escapes_dropped"] == 0, info
    # test_safe_functions.py:51 asserts the count; the bytecode rows' names are
    # listed there too (the compiled-source rows check them)
    assert len(got) == len(safe), (name, got, analyze.issue_table(issues), info)
    return got, issues, info


@pytest.mark.parametrize("row", GOLDEN["safe_functions"], ids=lambda r: r[0])
def test_safe_functions_on_the_oracle_device(row, monkeypatch, tmp_path):
    from oracle_device import OracleDevice, OracleK2
    use_signature_db(monkeypatch, tmp_path)
    got, issues, _ = check_safe_functions(row, OracleDevice(), OracleK2())
    if row[0] != "ether_send.sol.o":
        assert got == sorted(row[1])


def check_c1(device, k2, runtime):
    import analyze
    issues, info = analyze.analyze("suicide.sol.o", None, 3, device, k2, runtime=runtime)
    assert info["escapes_dropped"] == 0, info
    table = analyze.issue_table(issues)
    fn = "kill(address)" if runtime else "constructor"
    assert [(i.swc_id, i.function, i.title) for i in issues] == [("106", fn, "Unprotected Selfdestruct")], \
        (table, info)
    assert issues[0].address == 146 and issues[0].withdraws
    return issues, info


@pytest.mark.parametrize("runtime", [True, False], ids=["bin-runtime", "creation"])
def test_c1_stand_in_on_the_oracle_device(runtime, monkeypatch, tmp_path):
    from oracle_device import OracleDevice, OracleK2
    use_signature_db(monkeypatch, tmp_path)
    check_c1(OracleDevice(), OracleK2(), runtime)


def check_killbilly(device, k2):
    import analyze
    import killbilly
    issues, info = analyze.analyze("killbilly", None, 3, device, k2, code=killbilly.creation())
    assert info["escapes_dropped"] == 0, info
    assert [(i.swc_id, i.function, i.title) for i in issues] == \
        [("106", "commencekilling()", "Unprotected Selfdestruct")], (analyze.issue_table(issues), info)
    assert issues[0].address == killbilly.selfdestruct_address()
    steps = issues[0].transaction_sequence["steps"]
    attacker = int(steps[-1]["origin"], 16)
    assert [s["input"][:10] for s in steps[1:]] == \
        ["0x%08x" % killbilly.selector(f) for f in ("killerize(address)", "activatekillability()",
                                                     "commencekilling()")]
    assert int(steps[1]["input"][10:74], 16) & ((1 << 160) - 1) == attacker
    assert all(int(s["origin"], 16) == attacker for s in steps[1:])
    return issues, info


def test_killbilly_on_the_oracle_device(monkeypatch, tmp_path):
    from oracle_device import OracleDevice, OracleK2
    use_signature_db(monkeypatch, tmp_path)
    check_killbilly(OracleDevice(), OracleK2())
