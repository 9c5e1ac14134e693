"""The statespace graph (svm.py:549-637, cfg.py) on a device: a symbolic
message call run by a LaserEVM with requires_statespace (every state stepped
one instruction at a time, manage_cfg per step) against the same call run by
the batched core without it.  Shared by test_statespace_cpu.py (oracle device)
and test_gpu_statespace.py (MI355X)."""
from __future__ import annotations

from collections import Counter

import symcases
import symref
from mythril_amd.laser import (BreadthFirstSearchStrategy, Disassembly, JumpType, LaserEVM, NodeFlags,
                               execute_symbolic_message_call, tx_id_manager)
from mythril_amd.laser.state import Account, WorldState
from mythril_amd.smt import solver

CONTRACTS = ("overflow.sol.o", "exceptions.sol.o", "symjump")

# PUSH1 0 CALLDATALOAD PUSH1 12 JUMPI  PUSH1 1 PUSH1 0 SSTORE STOP  JUMPDEST(12) PUSH1 2 PUSH1 0 SSTORE STOP
BRANCH = bytes.fromhex("600035600c57600160005500" "5b600260005500")
BRANCH_PCS = {"tx": [0, 1, 2, 3], "fall": [4, 5, 6, 7], "jump": [8, 9, 10, 11, 12]}


def run(device, name, statespace: bool, monkeypatch, code: bytes = None, signals: bool = False):
    """One symbolic message call (transaction id 1) into `name` (or `code`);
    returns (outcomes, laser): the transaction-end and world-state events
    of the laser and of the escape engine, as symcases counts them.  With
    `signals` the engine raises the transaction-end signals (world states are
    then the laser's open states, as in tests/analyze.py)."""
    monkeypatch.setattr(solver.args, "pruning_factor", 0)
    if code is None:
        ws, addr = symcases.deploy(device, name)
    else:
        ws = WorldState()
        ws.put_account(Account(symcases.CREATOR, balances=None))
        acct = Account(symcases.workloads.CONTRACT, code=Disassembly(code), concrete_storage=True)
        acct.contract_name = name
        ws.put_account(acct)
        addr = symcases.workloads.CONTRACT
    eng = symref.Engine(signals=signals)
    laser = LaserEVM(requires_statespace=statespace, device=device, strategy=BreadthFirstSearchStrategy,
                     execution_timeout=0, escape_handler=eng.step)
    got = Counter()
    laser.register_laser_hooks("transaction_end", lambda s, tx, ret, revert: got.update(
        [("txend", bool(revert), tuple(x.raw for x in s.world_state.constraints),
          s.environment.active_function_name)]))
    laser.register_laser_hooks("add_world_state", lambda s: got.update(
        [("ws", tuple(x.raw for x in s.world_state.constraints))]))
    laser.open_states = [ws]
    tx_id_manager.set_counter(0)
    execute_symbolic_message_call(laser, addr)
    got += symcases._outcomes_of_restatement(eng)
    return got, laser


def check_graph(laser) -> dict:
    """The graph's invariants as svm.py builds it; returns counts by edge type.
    * every edge joins two registered nodes (the first transaction's node has
      no predecessor);
    * a node's states are its straight-line instructions: consecutive pcs,
      every one but the last neither a JUMP nor a JUMPI (those end nodes);
    * a CONDITIONAL edge's target starts at a JUMPDEST or right after a JUMPI,
      and carries the successor's last path constraint (True on a concrete branch);
    * a node entered at a dispatcher entry has FUNC_ENTRY and its name."""
    nodes, edges = laser.nodes, laser.edges
    assert nodes and edges
    kinds = Counter(e.type for e in edges)
    for e in edges:
        assert e.node_to in nodes and e.node_from in nodes
    targets = {e.node_to for e in edges}
    # each node holds its own snapshot per instruction, never a live state
    ids = [id(s) for n in nodes.values() for s in n.states]
    assert len(ids) == len(set(ids))
    assert not any(s in laser.work_list for n in nodes.values() for s in n.states)
    for uid, n in nodes.items():
        pcs = [s.mstate.pc for s in n.states]
        assert pcs == list(range(pcs[0], pcs[0] + len(pcs))), (n.function_name, pcs)
        ins = n.states[0].environment.code.instruction_list
        for pc in pcs[:-1]:
            assert ins[pc]["opcode"] not in ("JUMP", "JUMPI")
        assert all(s.node is n for s in n.states)
        if uid in targets:
            first = ins[pcs[0]]
            into = [e for e in edges if e.node_to == uid]
            assert len(into) == 1
            if into[0].type == JumpType.CONDITIONAL:
                assert first["opcode"] == "JUMPDEST" or ins[pcs[0] - 1]["opcode"] == "JUMPI"
                cons = n.states[0].world_state.constraints
                cond = into[0].condition
                # a concrete branch's condition simplifies to True (instructions.py:1587)
                assert cond.is_true or cond is cons[-1] or cond.raw is cons[-1].raw
            code = n.states[0].environment.code
            if first["address"] in code.address_to_function_name:
                assert n.flags & NodeFlags.FUNC_ENTRY
                assert n.function_name == code.address_to_function_name[first["address"]]
        d = n.get_cfg_dict()
        assert d["code"].count("\\n") == len(n.states)
    return dict(kinds)


def shape(laser):
    """The graph as plain data, nodes in creation order: (contract, function,
    pcs, flags) per node, (type, from, to, condition term) per edge."""
    order = {uid: k for k, uid in enumerate(laser.nodes)}
    nodes = [(n.contract_name, n.function_name, tuple(s.mstate.pc for s in n.states), int(n.flags))
             for n in laser.nodes.values()]
    edges = [(e.type, order.get(e.node_from), order[e.node_to],
              None if e.condition is None else e.condition.raw) for e in laser.edges]
    return nodes, edges
