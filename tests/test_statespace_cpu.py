"""The statespace graph on the oracle device (svm.py:549-637,
transaction/symbolic.py:221-243, cfg.py).

* A hand-checked program: one symbolic JUMPI gives three nodes -- the
  transaction's, the fall-through's and the jump target's -- joined by two
  CONDITIONAL edges whose conditions are the successors' branch constraints.
* Reference contracts: the graph-building run (every state stepped one
  instruction at a time) ends the call in exactly the batched core's outcomes
  (transaction ends with their constraints and function names, world states,
  total states), and its nodes and edges satisfy the invariants svm.py builds
  them with (statespace_cases.check_graph).
* A second transaction joins the first's end node by a Transaction edge.

Parity against the reference's own graph is unpinned: z3 is absent, so the
reference cannot run here, and its outputs_expected/*.graph.html come from an
older Mythril."""
import pytest

import statespace_cases as sc
from mythril_amd.laser import JumpType
from oracle_device import OracleDevice


def test_branch_program_graph(monkeypatch):
    got, laser = sc.run(OracleDevice(), "Branch", True, monkeypatch, code=sc.BRANCH)
    nodes = list(laser.nodes.values())
    assert len(nodes) == 3 and len(laser.edges) == 2
    by_pcs = {tuple(s.mstate.pc for s in n.states): n for n in nodes}
    assert set(by_pcs) == {tuple(v) for v in sc.BRANCH_PCS.values()}
    tx = by_pcs[tuple(sc.BRANCH_PCS["tx"])]
    assert all(e.node_from == tx.uid and e.type == JumpType.CONDITIONAL for e in laser.edges)
    assert {e.node_to for e in laser.edges} == {n.uid for n in nodes if n is not tx}
    assert all(n.contract_name == "Branch" for n in nodes)
    # the two conditions are the two sides of the one symbolic branch
    conds = {e.node_to: e.condition for e in laser.edges}
    fall = by_pcs[tuple(sc.BRANCH_PCS["fall"])]
    jump = by_pcs[tuple(sc.BRANCH_PCS["jump"])]
    assert conds[fall.uid].raw is fall.states[0].world_state.constraints[-1].raw
    assert conds[jump.uid].raw is jump.states[0].world_state.constraints[-1].raw
    assert conds[fall.uid].raw is not conds[jump.uid].raw
    assert "0 PUSH1 0x00\\n2 CALLDATALOAD\\n" in tx.get_cfg_dict()["code"]
    sc.check_graph(laser)
    plain, _ = sc.run(OracleDevice(), "Branch", False, monkeypatch, code=sc.BRANCH)
    assert got == plain


@pytest.mark.parametrize("name", sc.CONTRACTS)
def test_graph_run_equals_the_batched_run(name, monkeypatch):
    got, laser = sc.run(OracleDevice(), name, True, monkeypatch)
    plain, laser0 = sc.run(OracleDevice(), name, False, monkeypatch)
    assert sum(got.values()) > 0
    assert got == plain
    assert laser.total_states == laser0.total_states
    assert laser0.nodes == {} and laser0.edges == []
    kinds = sc.check_graph(laser)
    assert kinds.get(JumpType.CONDITIONAL, 0) > 0


def test_second_transaction_joins_by_a_transaction_edge(monkeypatch):
    from mythril_amd.laser import execute_symbolic_message_call
    got, laser = sc.run(OracleDevice(), "Branch", True, monkeypatch, code=sc.BRANCH, signals=True)
    ends = list(laser.open_states)
    assert len(ends) == 2 and all(ws.node is not None for ws in ends)
    n_nodes = len(laser.nodes)
    execute_symbolic_message_call(laser, sc.symcases.workloads.CONTRACT)
    tx_edges = [e for e in laser.edges if e.type == JumpType.Transaction]
    assert len(tx_edges) == 2
    assert {e.node_from for e in tx_edges} == {ws.node.uid for ws in ends}
    assert len(laser.nodes) == n_nodes + 2 * 3
    sc.check_graph(laser)


def test_graph_shape_is_deterministic(monkeypatch):
    """Two runs build the same graph (what test_gpu_statespace.py compares
    across devices)."""
    a = sc.shape(sc.run(OracleDevice(), "exceptions.sol.o", True, monkeypatch)[1])
    b = sc.shape(sc.run(OracleDevice(), "exceptions.sol.o", True, monkeypatch)[1])
    assert a == b and len(a[0]) > 3


@pytest.mark.parametrize("name", ["overflow.sol.o", "exceptions.sol.o"])
def test_graph_run_filters_forks_as_the_batched_run(name, monkeypatch):
    """Two transactions with the fork filter and the per-transaction
    reachability filter on (pruning factor 1, kernel 2 on bv_ref, witness
    seeds): the graph run -- svm.py's loop one state and one instruction at a
    time -- and the batched run answer the same queries the same way, leave the
    model cache's LRU in the same order and end the same paths in the same
    order (the batched core's event order is the literal loop's, §3.3)."""
    import test_fork_batch_cpu as fb
    from mythril_amd.laser import LaserEVM

    class GraphLaser(LaserEVM):
        def __init__(self, *args, **kwargs):
            kwargs["requires_statespace"] = True
            super().__init__(*args, **kwargs)
    try:
        ends_a, lru_a, fs_a, st_a, _, open_a = fb._run(name, True, monkeypatch)
        monkeypatch.setattr(fb, "LaserEVM", GraphLaser)
        ends_b, lru_b, fs_b, st_b, _, open_b = fb._run(name, True, monkeypatch)
    finally:
        fb.keccak_function_manager.reset()
        fb.tx_id_manager.restart_counter()
        fb.solver.get_model.cache_clear()
    assert ends_a == ends_b and open_a == open_b
    assert lru_a == lru_b
    for k in ("queries", "kept", "pruned", "unknown"):
        assert fs_a[k] == fs_b[k]
    assert st_a == st_b
    assert fs_a["queries"] > 10


@pytest.mark.parametrize("strategy", ["bfs", "delayed"])
@pytest.mark.parametrize("row", __import__("test_integration_cpu").GOLDEN["issue_counts"],
                         ids=lambda r: f"{r[0]}-{r[1]}")
def test_analysis_rows_with_the_graph(row, strategy, monkeypatch, tmp_path):
    """analysis_tests.py's rows with requires_statespace set (as SymExecWrapper
    sets it for POST modules), under BFS and --strategy delayed (whose drains
    the graph run steps one state at a time): the reference's count and the
    same SWC ids and functions as the batched run (test_integration_cpu.check_row)."""
    import test_integration_cpu as ti
    from fnames import use_signature_db
    from oracle_device import OracleK2
    use_signature_db(monkeypatch, tmp_path)
    ti.check_row(row, OracleDevice(), OracleK2(), strategy=strategy, statespace=True)
