"""ModelCache.conjunct_rows keeps rows per pool generation (_RowGen): the same
non-seed models and the same seed list at one completion epoch, in any order.
Rows served from a generation must equal evaluating the conjuncts afresh on the
pool as given (kernel 2's oracle here); only conjuncts new to the generation are
evaluated; a new epoch, a changed head or a pool of other models (the search's
candidates) is evaluated again."""
import numpy as np

from mythril_amd.smt import solver
from mythril_amd.smt.expr import UGT, ULT, Function, symbol_factory
from mythril_amd.smt.program import FuncInterp
from mythril_amd.smt.solver import Model, ModelRef
from oracle_device import OracleK2


class _Seeds:
    """The WitnessSeeds surface the cache reads: models(), epoch, revision()."""

    def __init__(self, n=150, seed=7):
        rng = np.random.default_rng(seed)
        self.assign = [{"x": int(a), "y": int(b), "f": FuncInterp(0, {})}
                       for a, b in zip(rng.integers(0, 16, n), rng.integers(0, 4, n))]
        self._models = [Model([ModelRef(a)]) for a in self.assign]
        for m, a in zip(self._models, self.assign):
            m.raw[0].assignment = a               # shared, as WitnessSeeds completes in place
        self.epoch = 1

    def models(self):
        return self._models

    def revision(self, name):
        return self.epoch


def _head(n=12, seed=11):
    rng = np.random.default_rng(seed)
    return [Model([ModelRef({"x": int(a), "y": int(b)})]) for a, b in zip(rng.integers(0, 16, n), rng.integers(0, 4, n))]


def _conjuncts():
    x = symbol_factory.BitVecSym("x", 256)
    y = symbol_factory.BitVecSym("y", 256)
    k = symbol_factory.BitVecVal
    f = Function("f", [256], 256)
    return [UGT(x, k(5, 256)).raw, (x + y == k(7, 256)).raw, ULT(y, k(2, 256)).raw, (x != y).raw,
            (f(x) == k(42, 256)).raw]


def _bits(row, n):
    return np.unpackbits(row.view(np.uint8), bitorder="little")[:n]


def _fresh(conjuncts, pool):
    return solver.ModelCache(device=OracleK2()).conjunct_rows(conjuncts, pool)


def _cache():
    mc = solver.ModelCache(device=OracleK2())
    mc.seed_source = _Seeds()
    mc._seed_models()
    return mc


def _same(got, want, n):
    assert set(got) == set(want)
    for c in want:
        assert np.array_equal(_bits(got[c], n), _bits(want[c], n)), c
        assert len(got[c]) == len(want[c])


def test_permuted_pool_is_served_from_the_generation():
    mc = _cache()
    head = _head()
    cs = _conjuncts()
    pool = head + mc.seeds
    _same(mc.conjunct_rows(cs, pool), _fresh(cs, pool), len(pool))
    launches, evals = mc.launches, mc.part_evals
    perm = head[::-1][3:] + head[::-1][:3]          # LRU moves reorder the head
    pool2 = perm + mc.seeds
    _same(mc.conjunct_rows(cs, pool2), _fresh(cs, pool2), len(pool2))
    assert (mc.launches, mc.part_evals) == (launches, evals)


def test_only_new_conjuncts_are_evaluated():
    mc = _cache()
    head = _head()
    cs = _conjuncts()
    pool = head + mc.seeds
    mc.conjunct_rows(cs[:2], pool)
    evals = mc.part_evals
    got = mc.conjunct_rows(cs, head[1:] + head[:1] + mc.seeds)
    assert mc.part_evals - evals == (len(cs) - 2) * len(pool)
    _same(got, _fresh(cs, head[1:] + head[:1] + mc.seeds), len(pool))


def test_a_new_epoch_or_head_is_evaluated_again():
    mc = _cache()
    head = _head()
    cs = _conjuncts()
    mc.conjunct_rows(cs, head + mc.seeds)
    # completion adds interpretation entries to the seeds in place, with a new
    # epoch (WitnessSeeds._complete: keccak256_N, Power)
    src = mc.seed_source
    for a in src.assign[:40]:
        a["f"].entries[(a["x"],)] = 42
    src.epoch += 1
    launches = mc.launches
    pool = head + mc.seeds
    _same(mc.conjunct_rows(cs, pool), _fresh(cs, pool), len(pool))
    assert mc.launches == launches + 1
    # a model the search found joins the head: another generation
    pool = head + _head(1, seed=99) + mc.seeds
    _same(mc.conjunct_rows(cs, pool), _fresh(cs, pool), len(pool))
    assert mc.launches == launches + 2


def test_pools_without_the_seed_tail_are_not_kept():
    mc = _cache()
    cands = _head(40, seed=5)
    cs = _conjuncts()
    mc.conjunct_rows(cs, cands)
    launches = mc.launches
    _same(mc.conjunct_rows(cs, cands), _fresh(cs, cands), len(cands))
    assert mc.launches == launches + 1
    assert not mc._rowgens
