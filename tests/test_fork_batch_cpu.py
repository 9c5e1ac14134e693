"""Batched fork filters (svm.py:319-326) and the per-transaction reachability
filter (svm.py:244-249) on CPU: the queries of consecutive MG_FORK events are
evaluated in one kernel-2 launch (here the bv_ref stand-in) and answered in the
reference's order, so every answer, the model cache's LRU order and the paths
that survive equal the one-query-per-fork loop; witness seeds answer queries
the LRU cannot (a seed is a model of the whole query, keccak axioms included).
"""
import pytest

import symcases
import symref
from mythril_amd import workloads
from mythril_amd.laser import BreadthFirstSearchStrategy, LaserEVM
from mythril_amd.laser.transaction import tx_id_manager
from mythril_amd.laser.witness import WitnessSeeds, dispatch_selectors
from mythril_amd.smt import solver
from mythril_amd.smt.keccak_manager import keccak_function_manager
from mythril_amd.smt.solver import ModelCache
from oracle_device import OracleDevice, OracleK2


@pytest.fixture(autouse=True)
def _clean_globals():
    yield
    keccak_function_manager.reset()
    tx_id_manager.restart_counter()
    solver.get_model.cache_clear()


def _run(name, batched, monkeypatch, n_seeds=48):
    keccak_function_manager.reset()
    tx_id_manager.restart_counter()
    solver.get_model.cache_clear()
    k2 = OracleK2()
    mc = ModelCache(device=k2)
    monkeypatch.setattr(solver, "model_cache", mc)
    code = workloads.bytecode(name)
    ws, addr = symcases.deploy(OracleDevice(), name)
    seeds = WitnessSeeds([code], n=n_seeds, storage_names=[f"Storage{addr}"])
    mc.seed_source = seeds
    eng = symref.Engine()

    def handler(st):
        try:
            return eng.step(st)
        except symref.Unsupported:
            return []
    laser = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=BreadthFirstSearchStrategy, transaction_count=2,
                     execution_timeout=0, escape_handler=handler)
    laser.unknown_forks = "keep"
    if not batched:
        def one_by_one(s, new_states, track_gas, final_states):
            laser._filter_fork(new_states)
            laser.work_list.extend(new_states)
            laser.total_states += len(new_states)
        laser._queue_fork = one_by_one
    ends = []
    laser.register_laser_hooks("transaction_end", lambda s, tx, ret, revert: ends.append(
        (bool(revert), tuple(x.raw for x in s.world_state.constraints))))
    laser.open_states = [ws]
    laser.execute_transactions(addr)
    pool = seeds.models()
    lru = [pool.index(m) for m in mc.model_cache.lru_cache]
    return ends, lru, dict(laser.fork_stats), dict(mc.stats), k2.launches, len(laser.open_states)


@pytest.mark.parametrize("name", ["overflow.sol.o"])
def test_batched_fork_filters_equal_the_sequential_loop(name, monkeypatch):
    a = _run(name, True, monkeypatch)
    b = _run(name, False, monkeypatch)
    ends_a, lru_a, fs_a, st_a, launches_a, open_a = a
    ends_b, lru_b, fs_b, st_b, launches_b, open_b = b
    assert ends_a == ends_b and lru_a == lru_b and open_a == open_b
    for k in ("queries", "kept", "pruned", "unknown"):
        assert fs_a[k] == fs_b[k]
    assert st_a == st_b
    assert fs_a["queries"] > 10 and st_a["seed_hits"] > 0
    assert launches_a < launches_b               # groups share a launch


def test_witness_seeds_satisfy_the_keccak_axioms():
    """Every seed, completed for the registered inputs, satisfies the
    KeccakFunctionManager conjunct (keccak_function_manager.py:116-179)."""
    from mythril_amd.smt.expr import Concat, symbol_factory
    keccak_function_manager.reset()
    tx_id_manager.restart_counter()
    tx_id_manager.get_next_tx_id()
    code = workloads.bytecode("overflow.sol.o")
    assert 0xA3210E87 in dispatch_selectors(code)
    seeds = WitnessSeeds([code], n=16)
    sender = symbol_factory.BitVecSym("sender_1", 256)
    x = Concat(sender & symbol_factory.BitVecVal((1 << 160) - 1, 256), symbol_factory.BitVecVal(0, 256))
    keccak_function_manager.create_keccak(x)
    keccak_function_manager.create_keccak(symbol_factory.BitVecVal(7, 512))
    h = keccak_function_manager.create_keccak(Concat(keccak_function_manager.create_keccak(x),
                                                     symbol_factory.BitVecVal(1, 256)))
    assert h.symbolic
    cond = keccak_function_manager.create_conditions()
    for m in seeds.models():
        assert m.eval(cond.raw, model_completion=True).param == 1


def test_refuting_backend_prunes_and_counts_divergences(monkeypatch):
    """With a real (here: stub) backend installed the backend answers before the
    witness seeds (mythril_amd/smt/solver.py _seeds_first); an UNSAT prunes, a
    timeout prunes unless a seed satisfies the query -- then the path is kept
    and counted as a divergence."""
    import symcases
    import symref
    from test_gpu_fork_filter import StubBackend
    from mythril_amd import workloads
    from mythril_amd.laser import BreadthFirstSearchStrategy, LaserEVM
    from mythril_amd.laser.transaction import tx_id_manager
    from mythril_amd.smt.keccak_manager import keccak_function_manager
    keccak_function_manager.reset()
    tx_id_manager.restart_counter()
    solver.get_model.cache_clear()
    monkeypatch.setattr(solver.args, "pruning_factor", 1)
    mc = solver.ModelCache(device=OracleK2())
    monkeypatch.setattr(solver, "model_cache", mc)
    be = StubBackend()
    monkeypatch.setattr(solver, "solver_backend", be)
    name = "overflow.sol.o"
    ws, addr = symcases.deploy(OracleDevice(), name)
    mc.seed_source = WitnessSeeds([workloads.bytecode(name)], n=48, storage_names=[f"Storage{addr}"])
    eng = symref.Engine()
    laser = LaserEVM(requires_statespace=False, device=OracleDevice(), strategy=BreadthFirstSearchStrategy, transaction_count=2,
                     execution_timeout=0, escape_handler=lambda st: eng.step(st))
    laser.open_states = [ws]
    laser.execute_transactions(addr)
    assert be.calls > 0
    assert laser.fork_stats["pruned"] > 0
    assert mc.stats["divergences"] > 0, (laser.fork_stats, mc.stats)
    assert mc.stats["seed_hits"] == 0            # seeds never pre-empt a real backend
    solver.get_model.cache_clear()
