"""ModelCache.conjunct_rows derives a negated conjunct's bitmap from its
partner's (a JUMPI's two branch conditions: eq / distinct, X / not X) instead of
compiling and evaluating both; the rows must equal those of evaluating each on
its own (kernel 2's oracle here)."""
import numpy as np

from mythril_amd.smt import solver
from mythril_amd.smt.expr import Not, UGT, symbol_factory
from mythril_amd.smt.solver import Model, ModelRef
from oracle_device import OracleK2


def _pool(n=200, seed=3):
    rng = np.random.default_rng(seed)
    return [Model([ModelRef({"x": int(v), "y": int(w)})]) for v, w in zip(rng.integers(0, 12, n), rng.integers(0, 3, n))]


def test_negations_equal_separate_evaluation():
    x = symbol_factory.BitVecSym("x", 256)
    y = symbol_factory.BitVecSym("y", 256)
    c1 = UGT(x, symbol_factory.BitVecVal(5, 256)).raw
    c2 = Not(UGT(x, symbol_factory.BitVecVal(5, 256))).raw
    c3 = (x + y == symbol_factory.BitVecVal(7, 256)).raw
    c4 = (x + y != symbol_factory.BitVecVal(7, 256)).raw
    pool = _pool()
    together = solver.ModelCache(device=OracleK2()).conjunct_rows([c2, c1, c4, c3], pool)
    apart = {}
    for c in (c1, c2, c3, c4):
        apart.update(solver.ModelCache(device=OracleK2()).conjunct_rows([c], pool))
    n = len(pool)
    for c in (c1, c2, c3, c4):
        a = np.unpackbits(together[c].view(np.uint8), bitorder="little")[:n]
        b = np.unpackbits(apart[c].view(np.uint8), bitorder="little")[:n]
        assert np.array_equal(a, b), c
    # the pair's bits partition the pool, and nothing is set past it
    assert not (together[c1] & together[c2]).any()
    full = np.unpackbits((together[c3] | together[c4]).view(np.uint8), bitorder="little")
    assert full[:n].all() and not full[n:].any()


def test_one_of_each_pair_is_compiled():
    x = symbol_factory.BitVecSym("x", 256)
    c = (x == symbol_factory.BitVecVal(3, 256)).raw
    nc = (x != symbol_factory.BitVecVal(3, 256)).raw
    mc = solver.ModelCache(device=OracleK2())
    mc.conjunct_rows([c, nc], _pool())
    assert (c in mc._progs) != (nc in mc._progs)
