"""laser/witness.py's column evaluator (eval_all) against the per-model
reference evaluator (tests/smt_eval.py) on the table-shaped constraint sets of
test_smt_programs, with calldata held as dict entries and as dense bytes."""
from __future__ import annotations

import random

from mythril_amd.laser.witness import eval_all
from mythril_amd.smt.expr import And, Array, Concat, Extract, ZeroExt, symbol_factory
from mythril_amd.smt.program import ArrayInterp
from smt_eval import evaluate
from test_smt_programs import _random_table_constraints, _random_table_models

BVS, BVV = symbol_factory.BitVecSym, symbol_factory.BitVecVal


def test_eval_all_matches_the_reference_evaluator():
    rng = random.Random(99)
    sets = [_random_table_constraints(rng) for _ in range(60)]
    models = _random_table_models(random.Random(3), 40, None)
    for s in sets:
        root = And(*s).raw
        assert [bool(v) for v in eval_all(root, models)] == [bool(evaluate(root, m)) for m in models]


def test_eval_all_reads_dense_calldata_like_entries():
    cd = Array("1_calldata", 256, 8)
    i = BVS("i", 256)
    terms = [Concat(cd[BVV(0, 256)], cd[BVV(1, 256)], cd[BVV(2, 256)], cd[BVV(3, 256)]),
             ZeroExt(248, cd[i]), Extract(7, 0, ZeroExt(248, cd[BVV(40, 256)]))]
    rng = random.Random(5)
    dense, plain = [], []
    for m in range(50):
        data = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 70)))
        d = rng.choice([0, 0xAB])
        dense.append({"1_calldata": ArrayInterp(d, dense=data), "i": rng.randrange(0, 80)})
        plain.append({"1_calldata": ArrayInterp(d, dict(enumerate(data))), "i": dense[-1]["i"]})
    for t in terms:
        want = [evaluate(t.raw, m) for m in plain]
        assert list(eval_all(t.raw, dense)) == want == list(eval_all(t.raw, plain))
    assert all(m["1_calldata"].untouched_dense() is not None for m in dense)
