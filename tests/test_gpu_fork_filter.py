"""Kernel 2 at the engine's own feasibility call sites, on an MI355X (SURVEY §8
row K2.4): the fork filter (svm.py:319-326, `_filter_fork` / batched
`_flush_forks`) and the per-transaction reachability filter (svm.py:244-249)
with pruning on, driven by a symbolic `-t 2` run of reference bytecode on
kernel 1 (symbolic lanes) with kernel 2 answering every quick-sat query of
the model cache.

The same run with kernel 2 replaced by its C oracle (oracle/bv_ref.c behind
tests/oracle_device.OracleK2) is the checker: transaction ends with their
constraint sequences (device halts and escaped paths alike), the open states,
the fork-filter decisions (queries / kept / pruned / unknown), the model
cache's hit statistics and its final LRU order must be identical.
"""
from collections import Counter

import pytest

import symcases
import symref
from mythril_amd import workloads
from mythril_amd.device import GpuDevice
from mythril_amd.laser import BreadthFirstSearchStrategy, LaserEVM
from mythril_amd.laser.transaction import tx_id_manager
from mythril_amd.laser.witness import WitnessSeeds
from mythril_amd.smt import solver
from mythril_amd.smt.keccak_manager import keccak_function_manager
from mythril_amd.smt.solver import ModelCache
from oracle_device import OracleK2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


@pytest.fixture(autouse=True)
def _clean_globals():
    yield
    keccak_function_manager.reset()
    tx_id_manager.restart_counter()
    solver.get_model.cache_clear()


class _CountingK2:
    """GpuDevice's kernel-2 entry points with a launch count."""

    def __init__(self, dev):
        self.dev, self.launches = dev, 0

    def eval(self, prog, pool):
        self.launches += 1
        return self.dev.eval(prog, pool)

    def eval_bits(self, prog, pool):
        self.launches += 1
        return self.dev.eval_bits(prog, pool)


class StubBackend:
    """A stand-in SMT backend that refutes a fixed subset of queries: UNSAT
    when the query has an even number (at least 4) of leaf conjuncts, a solver
    timeout otherwise (constraints.py:35-38: a timeout prunes with the default timeout;
    get_model then tries the witness seeds, a counted divergence).  Decisions
    depend only on the query, so two runs that pose the same queries prune the
    same paths."""

    def __init__(self):
        self.calls = 0

    def __call__(self, constraints, minimize, maximize, timeout):
        from mythril_amd.smt.solver import SolverTimeOutException, UnsatError, _conjuncts, query_raw
        self.calls += 1
        n = len(_conjuncts(query_raw(constraints)))
        if n >= 4 and n % 2 == 0:
            raise UnsatError()
        raise SolverTimeOutException()


def _run(name, k1, k2, monkeypatch, n_seeds=48, backend=None):
    keccak_function_manager.reset()
    tx_id_manager.restart_counter()
    solver.get_model.cache_clear()
    monkeypatch.setattr(solver.args, "pruning_factor", 1)
    mc = ModelCache(device=k2)
    monkeypatch.setattr(solver, "model_cache", mc)
    if backend is not None:
        monkeypatch.setattr(solver, "solver_backend", backend)
    code = workloads.bytecode(name)
    ws, addr = symcases.deploy(k1, name)
    seeds = WitnessSeeds([code], n=n_seeds, storage_names=[f"Storage{addr}"])
    mc.seed_source = seeds
    eng = symref.Engine()

    def handler(st):
        try:
            return eng.step(st)
        except symref.Unsupported:
            return []
    laser = LaserEVM(requires_statespace=False, device=k1, strategy=BreadthFirstSearchStrategy, transaction_count=2,
                     execution_timeout=0, escape_handler=handler)
    laser.unknown_forks = "keep"
    ends = []
    laser.register_laser_hooks("transaction_end", lambda s, tx, ret, revert: ends.append(
        (bool(revert), tuple(x.raw for x in s.world_state.constraints))))
    laser.open_states = [ws]
    laser.execute_transactions(addr)
    ends += [(kind == "revert", tuple(x.raw for x in st.world_state.constraints)) for kind, st in eng.ended]
    pool = seeds.models()
    lru = [pool.index(m) for m in mc.model_cache.lru_cache]
    opened = Counter(tuple(x.raw for x in w.constraints) for w in laser.open_states)
    return {"ends": ends, "lru": lru, "forks": dict(laser.fork_stats), "cache": dict(mc.stats),
            "open": opened, "lane_steps": int(laser.lane_steps), "device_evals": mc.device_evals}


@pytest.mark.parametrize("name", ["overflow.sol.o", "exceptions.sol.o"])
def test_fork_and_reachability_filters_on_kernel2_equal_the_oracles(dev, name, monkeypatch):
    k2 = _CountingK2(dev)
    got = _run(name, dev, k2, monkeypatch)
    want = _run(name, dev, OracleK2(), monkeypatch)
    for key in ("ends", "open", "forks", "cache", "lru", "lane_steps"):
        assert got[key] == want[key], key
    # the filters really ran on kernel 2, with pruning on
    assert k2.launches > 0 and got["device_evals"] > 0
    assert got["forks"]["queries"] > 10 and got["cache"]["queries"] > 10
    assert got["lane_steps"] > 100 and len(got["ends"]) > 10


@pytest.mark.parametrize("name", ["overflow.sol.o", "exceptions.sol.o"])
def test_prunes_with_a_refuting_backend_equal_the_oracles(dev, name, monkeypatch):
    """with a backend that refutes (UNSAT) and times out on a
    known subset, the fork and reachability filters really prune, kernel 2 still
    answers what the LRU and the seeds can, and every decision, end and open
    state equals the run with kernel 2's C oracle.  Seeds are consulted only
    where the backend timed out (counted as divergences from the reference)."""
    got = _run(name, dev, _CountingK2(dev), monkeypatch, backend=StubBackend())
    want = _run(name, dev, OracleK2(), monkeypatch, backend=StubBackend())
    for key in ("ends", "open", "forks", "cache", "lru", "lane_steps"):
        assert got[key] == want[key], key
    assert got["forks"]["pruned"] > 0
    assert got["cache"]["divergences"] == want["cache"]["divergences"]
