"""Host side of the kernel-2 path (mythril_amd/smt/solver.py, keccak_manager.py) on CPU:
LRU / ModelCache bookkeeping, get_model's error behaviour, Constraints.is_possible,
and the keccak conjuncts — compiled for the device and evaluated by the oracle
and by the pure-Python restatement."""
import random

import pytest

from mythril_amd.keccak import keccak256
from mythril_amd.smt import solver
from mythril_amd.smt.expr import And, Concat, ULT, symbol_factory
from mythril_amd.smt.flatten import compile_sets
from mythril_amd.smt.keccak_manager import (INTERVAL_DIFFERENCE, PART, TOTAL_PARTS,
                                            KeccakFunctionManager)
from mythril_amd.smt.program import FuncInterp, ModelPool
from mythril_amd.smt.solver import (Constraints, LRUCache, Model, ModelCache, SolverTimeOutException,
                                    UnsatError, get_model)
from oracle.bv_ref import eval_batch
from smt_eval import evaluate

BVS, BVV = symbol_factory.BitVecSym, symbol_factory.BitVecVal


def test_lru_cache_semantics():
    c = LRUCache(2)
    c.put("a", 1)
    c.put("b", 1)
    assert c.get("a") == 1                  # a becomes most recent
    c.put("c", 1)                           # evicts the least recent: b
    assert list(c.lru_cache) == ["a", "c"]
    assert c.get("b") == -1


class _Backend:
    def __init__(self, result=None, exc=None):
        self.calls, self.result, self.exc = [], result, exc

    def __call__(self, constraints, minimize, maximize, timeout):
        self.calls.append((tuple(constraints), minimize, maximize, timeout))
        if self.exc:
            raise self.exc
        return self.result


@pytest.fixture
def fresh(monkeypatch):
    monkeypatch.setattr(solver, "model_cache", ModelCache(device=object()))
    yield
    solver.set_solver_backend(solver._no_backend)


def test_get_model_paths(fresh):
    x = BVS("x", 256)
    m = Model({"x": 3})
    be = _Backend(result=m)
    solver.set_solver_backend(be)
    with pytest.raises(UnsatError):
        get_model((ULT(x, BVV(5, 256)), False))
    # empty model cache: quick-sat cannot answer, the backend does; its model is cached
    assert get_model((ULT(x, BVV(5, 256)),)) is m
    assert list(solver.model_cache.model_cache.lru_cache.items()) == [(m, 1)]
    # minimize bypasses quick-sat
    get_model((ULT(x, BVV(6, 256)),), minimize=(x,))
    assert len(be.calls) == 2 and be.calls[1][1] == (x,)
    # lru_cache(2**23): the same query is answered without a new backend call
    get_model((ULT(x, BVV(5, 256)),))
    assert len(be.calls) == 2
    solver.time_handler.start_execution(0)
    try:
        with pytest.raises(UnsatError):
            get_model((ULT(x, BVV(7, 256)),))
    finally:
        solver.time_handler._start = None


def test_constraints_is_possible_error_mapping(fresh):
    x = BVS("x", 256)
    solver.set_solver_backend(_Backend(exc=SolverTimeOutException()))
    c = Constraints([ULT(x, BVV(9, 256))])
    assert c.is_possible() is False                 # default timeout -> False
    assert c.is_possible(solver_timeout=10) is True  # custom timeout -> True
    solver.set_solver_backend(_Backend(exc=UnsatError()))
    assert c.is_possible() is False
    assert c.get_model() is None
    c2 = c + [True]
    assert len(c2) == 2 and hash(c2.copy()) == hash(c2)
    assert Constraints([False]).is_possible() is False


def test_missing_backend_is_loud_not_a_prune(fresh):
    """Without an SMT backend a quick-sat miss raises SolverBackendMissing; it is
    never turned into is_possible() == False (a silent prune)."""
    x = BVS("x", 256)
    solver.set_solver_backend(solver._no_backend)
    c = Constraints([x == BVV(11, 256)])       # no built-in witness (variables 0) satisfies it
    with pytest.raises(solver.SolverBackendMissing):
        c.is_possible()
    with pytest.raises(solver.SolverBackendMissing):
        c.get_model()
    assert not issubclass(solver.SolverBackendMissing, (SolverTimeOutException, UnsatError))
    # what the built-in backend does decide: folded True / False, concrete keccak axioms
    assert Constraints([]).is_possible() is True
    assert Constraints([x == x]).is_possible() is True
    from mythril_amd.smt.keccak_manager import keccak_function_manager as km
    km.reset()
    h = km.create_keccak(BVV(0x1234, 256))
    assert Constraints([h == h]).is_possible() is True          # f(c) == keccak(c) witness


def test_keccak_manager_reference_behaviour():
    km = KeccakFunctionManager()
    assert km.get_empty_keccak_hash().value == int.from_bytes(keccak256(b""), "big")
    c = BVV(0xDEADBEEF, 256)
    h = km.create_keccak(c)
    assert h.value == int.from_bytes(keccak256((0xDEADBEEF).to_bytes(32, "big")), "big")
    x = BVS("x", 256)
    fx = km.create_keccak(Concat(x, BVV(0, 256)))
    km.create_keccak(BVS("y", 256))
    assert fx.raw.op == "uf" and fx.raw.param[0] == "keccak256_512"
    # intervals in first-use order: 512-bit inputs got the first one
    assert km.interval_hook_for_size == {}
    km.create_conditions()
    assert km.interval_hook_for_size[512] == TOTAL_PARTS - 34534
    assert km.interval_hook_for_size[256] == TOTAL_PARTS - 34534 - INTERVAL_DIFFERENCE


def test_keccak_conjunct_compiles_and_matches_python():
    km = KeccakFunctionManager()
    x, s = BVS("x", 256), BVS("slot", 256)
    km.create_keccak(BVV(7, 256))
    km.create_keccak(Concat(BVV(1, 256), BVV(2, 256)))
    fx = km.create_keccak(Concat(x, s))
    cond = km.create_conditions()
    sets = [[cond], [cond, ULT(fx, BVV(1 << 255, 256))]]
    prog, kept = compile_sets(sets)
    assert kept == [0, 1]
    lo = (TOTAL_PARTS - 34534) * PART
    rng = random.Random(3)
    h7 = int.from_bytes(keccak256((7).to_bytes(32, "big")), "big")
    h12 = int.from_bytes(keccak256((1).to_bytes(32, "big") + (2).to_bytes(32, "big")), "big")
    models = []
    for k in range(40):
        xv, sv = rng.getrandbits(256), rng.choice([0, 1, rng.getrandbits(256)])
        key = (xv << 256) | sv
        hv = (lo + 63) // 64 * 64 + 64 * rng.randrange(1 << 20) if k % 3 else rng.getrandbits(256)
        good = k % 4 != 0
        models.append({
            "x": xv, "slot": sv,
            "keccak256_256": FuncInterp(0, {(7,): h7}),
            "keccak256_256-1": FuncInterp(0, {(h7,): 7 if good else 8}),
            "keccak256_512": FuncInterp(0, {(key,): hv, ((1 << 256) | 2,): h12}),
            "keccak256_512-1": FuncInterp(0, {(hv,): key, (h12,): (1 << 256) | 2}),
        })
    pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables)
    fs, sc = eval_batch(prog, pool)
    for d, s_ in enumerate(sets):
        vals = [evaluate(And(*s_).raw, m) for m in models]
        assert (next((i for i, v in enumerate(vals) if v), 0xFFFFFFFF), sum(vals)) == (fs[d], sc[d])
    assert 0 < sc[0] < len(models)


def test_prefetched_bitmaps_survive_an_lru_eviction(monkeypatch):
    """a prefetch window's bitmaps place models by id().  When
    a backend miss inside the window evicts the LRU's oldest model, a model
    created afterwards must not inherit the dead model's bit: the entry keeps its
    pool alive, so the evicted model's id stays taken and quick-sat answers
    exactly as without the prefetch."""
    import gc
    import weakref
    from oracle_device import OracleK2
    mc = ModelCache(device=OracleK2())
    monkeypatch.setattr(solver, "model_cache", mc)
    x = BVS("x", 256)
    olds = [Model({"x": v}) for v in range(100)]
    for m in olds:
        mc.put(m, 1)
    key = ULT(x, BVV(1, 256)).raw                 # only x == 0 (the LRU's oldest) satisfies it
    mc.prefetch([key])
    oldest = weakref.ref(olds[0])
    del olds, m
    mc.put(Model({"x": 500}), 1)                  # a backend miss in the window evicts x == 0
    gc.collect()
    assert oldest() is not None                   # held by the prefetched entry, id not reusable
    fresh_models = [Model({"x": 1000 + k}) for k in range(200)]
    for fm in fresh_models[:99]:
        mc.put(fm, 1)
    assert mc.check_quick_sat(key) is False       # no model in the LRU satisfies x < 1
    mc.clear_prefetch()
    gc.collect()
    assert oldest() is None                       # released with the window
