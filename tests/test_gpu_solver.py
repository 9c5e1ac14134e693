"""ModelCache.check_quick_sat on kernel 2 (MI355X) against a pure-Python replay of
support_utils.py:60-68: the same model returned, the same LRU order afterwards,
for sequential calls and for the one-launch batch replay (mg_eval_bits)."""
import random

import pytest

from mythril_amd.device import GpuDevice
from mythril_amd.smt import solver
from mythril_amd.smt.expr import And
from mythril_amd.smt.solver import Model, ModelCache, get_model
from smt_eval import evaluate
from test_smt_programs import (_random_constraints, _random_table_constraints,
                               _random_table_models)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


def _queries_and_models(seed, n_queries, n_models):
    rng = random.Random(seed)
    qs = []
    for k in range(n_queries):
        cs = _random_table_constraints(rng) if k % 2 else _random_constraints(rng, rng.randrange(1, 4))
        qs.append(And(*cs))
    qs += [qs[rng.randrange(len(qs))] for _ in range(n_queries // 4)]     # repeats hit the memo
    rng.shuffle(qs)
    dicts = _random_table_models(random.Random(seed + 1), n_models, None)
    mr = random.Random(seed + 2)
    for d in dicts:
        d["y"] = d["y"] if mr.random() < 0.5 else mr.getrandbits(64)
        d["z"] = mr.choice([0, 1, mr.getrandbits(256)])
        d["cd4"] = mr.getrandbits(8)
    return qs, [Model(d) for d in dicts]


class PyModelCache:
    """support_utils.ModelCache restated over Python evaluation (test oracle)."""

    def __init__(self, models):
        self.cache = solver.LRUCache(100)
        for m in models:
            self.cache.put(m, 1)
        self.memo = {}

    def check_quick_sat(self, expr):
        key = expr.raw
        if key in self.memo:
            return self.memo[key]
        res = False
        for m in reversed(self.cache.lru_cache.keys()):
            if evaluate(key, m.assignment):
                self.cache.put(m, self.cache.get(m) + 1)
                res = m
                break
        self.memo[key] = res
        return res


def _fill(mc, models):
    for m in models:
        mc.put(m, 1)


def test_check_quick_sat_sequential_and_batched_match_python(dev):
    qs, models = _queries_and_models(17, 120, 100)
    ref = PyModelCache(models)
    want = [ref.check_quick_sat(q) for q in qs]
    seq = ModelCache(device=dev)
    _fill(seq, models)
    got_seq = [seq.check_quick_sat(q) for q in qs]
    bat = ModelCache(device=dev)
    _fill(bat, models)
    got_bat = bat.check_quick_sat_many(qs)
    assert [id(x) if x else None for x in got_seq] == [id(x) if x else None for x in want]
    assert [id(x) if x else None for x in got_bat] == [id(x) if x else None for x in want]
    order = [id(m) for m in ref.cache.lru_cache]
    assert [id(m) for m in seq.model_cache.lru_cache] == order
    assert [id(m) for m in bat.model_cache.lru_cache] == order
    assert [seq.model_cache.lru_cache[m] for m in seq.model_cache.lru_cache] == \
        [ref.cache.lru_cache[m] for m in ref.cache.lru_cache]
    assert bat.launches == 1 and sum(1 for x in want if x) > 20


def test_get_model_answers_from_the_device_cache(dev, monkeypatch):
    qs, models = _queries_and_models(5, 20, 60)
    mc = ModelCache(device=dev)
    _fill(mc, models)
    monkeypatch.setattr(solver, "model_cache", mc)
    calls = []

    def backend(*a):
        calls.append(a)
        raise solver.UnsatError

    solver.set_solver_backend(backend)
    try:
        ref = PyModelCache(models)
        for q in qs:
            want = ref.check_quick_sat(q)
            if want:
                assert get_model((q,)) is want
            else:
                with pytest.raises(solver.UnsatError):
                    get_model((q,))
        assert calls and len(calls) < len(qs)
    finally:
        solver.set_solver_backend(solver._no_backend)


def test_multi_model_entries_use_their_last_internal_model(dev):
    """Cached models made of several internal models (the independence
    solver's, laser/smt/model.py) are evaluated by quick-sat under the last
    internal model: And has no declaration a model declares (model.py:45-59)."""
    from mythril_amd.smt.solver import ModelRef
    qs, singles = _queries_and_models(23, 60, 80)
    rng = random.Random(5)
    wrapped = [Model([ModelRef(rng.choice(singles).assignment), ModelRef(m.assignment)])
               for m in singles]
    ref = PyModelCache(wrapped)
    want = [ref.check_quick_sat(q) for q in qs]
    mc = ModelCache(device=dev)
    _fill(mc, wrapped)
    got = [mc.check_quick_sat(q) for q in qs]
    assert [id(m) if m else None for m in got] == [id(m) if m else None for m in want]
    assert sum(1 for m in want if m) > 5
    bat = ModelCache(device=dev)
    _fill(bat, wrapped)
    got_b = bat.check_quick_sat_many(qs)
    assert [id(m) if m else None for m in got_b] == [id(m) if m else None for m in want]
