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


def test_eval_all_calldata_words_read_the_bytes():
    """SymbolicCalldata words (the MG_SYM_CDLOAD concat of 32 guarded selects)
    evaluated from the seeds' bytes equal the per-byte semantics, at offsets
    inside, across and past the data, with sizes that disagree with the data's
    length, and at offsets past 2^255 (signed guard)."""
    from mythril_amd.laser.symbolic import SymbolicCalldata
    cd = SymbolicCalldata("9")
    o = BVS("o", 256)
    words = [cd.get_word_at(BVV(4, 256)), cd.get_word_at(BVV(60, 256)), cd.get_word_at(o),
             cd.get_word_at(o + BVV(4, 256))]
    rng = random.Random(11)
    dense, plain = [], []
    for m in range(120):
        data = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 4, 36, 68, 100])))
        size = len(data) if m % 3 else rng.choice([0, len(data) + 5, max(len(data) - 7, 0), (1 << 256) - 1])
        off = rng.choice([0, 3, 30, 64, 99, (1 << 255) + 2, (1 << 256) - 2])
        d = rng.choice([0, 0, 7])
        dense.append({"9_calldata": ArrayInterp(d, dense=data), "9_calldatasize": size, "o": off})
        plain.append({"9_calldata": ArrayInterp(d, dict(enumerate(data))), "9_calldatasize": size, "o": off})
    for w in words:
        want = [evaluate(w.raw, m) for m in plain]
        assert list(eval_all(w.raw, dense)) == want == list(eval_all(w.raw, plain))
