"""Symbolic transactions with the open world states sharded over ranks and
rebalanced at every transaction boundary (mythril_amd/laser/
sharded.py execute_symbolic_transactions), on CPU: gloo ranks, the oracle-backed
device, kernel 2's stand-in and witness seeds (no SMT backend: unknown fork
answers keep both paths, as in tests/test_fork_batch_cpu.py).

Against the single-process run of the same transactions:
* the union over ranks of the open world states is the same multiset (callee
  storage chain and path constraints, with each state's transaction ids
  renamed by their position in its own transaction sequence: ids are global
  positions, which may differ between the runs as §8(e) allows);
* every rank's coverage after the exchange is the single-process coverage and
  every rank's transaction-id counter the single-process counter;
* the states actually moved between ranks (rebalancing is exercised), and the
  keccak inputs each rank registered reached the others (the same distinct
  inputs on every rank, as many as the single process registered).
"""
import os
import re
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

NAME = "overflow.sol.o"
TX = 2
_ID = re.compile(r"(sender_|call_value|gas_price)(\d+)|(?<![\w])(\d+)(_calldata(?:size)?)")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _norm(text: str, ids) -> str:
    pos = {i: f"T{k}" for k, i in enumerate(ids)}

    def sub(m):
        if m.group(1):
            return m.group(1) + pos.get(m.group(2), "T?")
        return pos.get(m.group(3), "T?") + m.group(4)
    return _ID.sub(sub, text)


def _fingerprint(ws, addr):
    ids = [str(tx.id) for tx in ws.transaction_sequence]
    st = ws[addr].storage
    chain = repr(st.chain_raw()) if st.is_chain else repr(sorted(st.items()))
    cons = sorted(_norm(repr(c.raw), ids) for c in ws.constraints)
    return _norm(chain, ids), tuple(cons)


def _run():
    import symcases
    import symref
    from mythril_amd import workloads
    from mythril_amd.laser import BreadthFirstSearchStrategy, InstructionCoveragePlugin, LaserEVM
    from mythril_amd.laser.sharded import execute_symbolic_transactions, rebalance
    from mythril_amd.laser.transaction import tx_id_manager
    from mythril_amd.laser.witness import WitnessSeeds
    from mythril_amd.smt import solver
    from mythril_amd.smt.keccak_manager import keccak_function_manager
    from mythril_amd.smt.solver import ModelCache
    from oracle_device import OracleDevice, OracleK2

    keccak_function_manager.reset()
    tx_id_manager.restart_counter()
    solver.get_model.cache_clear()
    mc = ModelCache(device=OracleK2())
    solver.model_cache = mc
    ws, addr = symcases.deploy(OracleDevice(), NAME)
    mc.seed_source = WitnessSeeds([workloads.bytecode(NAME)], n=32, storage_names=[f"Storage{addr}"])
    eng = symref.Engine()

    def handler(st):
        """The restatement steps a symbolic state; a state it ends with STOP /
        RETURN / past the code ends its transaction as svm.py:452-460 does."""
        n = len(eng.ended)
        try:
            out = eng.step(st)
        except symref.Unsupported:
            return []
        for kind, s in eng.ended[n:]:
            if kind in ("stop", "return", "end"):
                for hook in vm._transaction_end_hooks:
                    hook(s, s.current_transaction, None, False)
                vm._add_world_state(s)
        return out
    vm = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=BreadthFirstSearchStrategy, transaction_count=TX,
                  execution_timeout=0, escape_handler=handler)
    vm.unknown_forks = "keep"
    cov = InstructionCoveragePlugin()
    cov.initialize(vm)
    vm.open_states = [ws]
    moved = []
    orig = rebalance.__globals__["rebalance"]

    def counting(laser):
        before = [id(s) for s in laser.open_states]
        counts = orig(laser)
        moved.append(sum(1 for s in laser.open_states if id(s) not in set(before)))
        return counts
    rebalance.__globals__["rebalance"] = counting
    try:
        execute_symbolic_transactions(vm, addr)
    finally:
        rebalance.__globals__["rebalance"] = orig
    prints = sorted(_fingerprint(s, addr) for s in vm.open_states)
    table = {k: list(v[1]) for k, v in vm.coverage().items()}
    n_inputs = sorted({repr(x.raw) for v in keccak_function_manager.symbolic_inputs.values() for x in v})
    return prints, table, tx_id_manager._next_transaction_id, sum(moved), n_inputs, vm.lane_steps


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out[rank] = _run()
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def single():
    return _run()


def test_single_process_symbolic_rounds(single):
    prints, table, counter, moved, n_inputs, steps = single
    assert len(prints) > 4 and counter > 2 and moved == 0


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_symbolic_rounds_equal_single_process(single, world):
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = [out[r] for r in range(world)]
    prints, table, counter, _, n_inputs, steps = single
    assert sorted(p for r in res for p in r[0]) == prints
    for r in res:
        assert r[1] == table and r[2] == counter
    assert sum(r[3] for r in res) > 0                    # states changed rank
    assert n_inputs and all(r[4] == res[0][4] for r in res)   # every rank knows every keccak input
    assert len(res[0][4]) == len(n_inputs)
    assert all(len(r[0]) > 0 for r in res)


def test_model_word_stream_round_trips():
    """exchange_models' u32 stream (sharded._models_to_words): ints, arrays and
    functions with multi-argument keys survive the trip."""
    from mythril_amd.laser.sharded import _models_to_words, _words_to_models
    from mythril_amd.smt.program import ArrayInterp, FuncInterp
    from mythril_amd.smt.solver import Model, ModelRef
    a = {"x": (1 << 256) - 1, "flag": 0, "1_calldata": ArrayInterp(7, {0: 0xA3, 5: 0}),
         "keccak256_512": FuncInterp(3, {((1 << 511) + 5,): 1 << 255}), "Power": FuncInterp(0, {(256, 2): 65536})}
    ms = [Model([ModelRef(a), ModelRef({"y": 12345})]), Model({"z": 1})]
    back = _words_to_models(_models_to_words(ms))
    assert len(back) == 2 and len(back[0].raw) == 2
    got = back[0].raw[0].assignment
    assert got["x"] == a["x"] and got["flag"] == 0
    assert got["1_calldata"].default == 7 and got["1_calldata"].entries == {0: 0xA3, 5: 0}
    assert got["keccak256_512"].entries == a["keccak256_512"].entries and got["Power"].entries == {(256, 2): 65536}
    assert back[0].raw[1].assignment == {"y": 12345} and back[1].raw[0].assignment == {"z": 1}
