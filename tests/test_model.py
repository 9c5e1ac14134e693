"""The model wrapper (laser/smt/model.py:6-59) on CPU: ModelRef.eval (z3 model.eval
by substitution + the builders' constant folding) against the test-side
evaluator tests/smt_eval.py on random constraint sets with arrays, uninterpreted
functions and 512-bit keys; multi-model lookup order; which internal model
quick-sat evaluates a conjunction under; keccak get_concrete_hash_data."""
import random

from mythril_amd.smt.expr import And, Function, Not, symbol_factory
from mythril_amd.smt.keccak_manager import KeccakFunctionManager
from mythril_amd.smt.program import FuncInterp
from mythril_amd.smt.solver import Model, ModelRef, _view
from smt_eval import evaluate
from test_smt_programs import _random_constraints, _random_table_constraints, _random_table_models

BVS = symbol_factory.BitVecSym
BVV = symbol_factory.BitVecVal


def test_eval_with_completion_matches_python_semantics():
    rng = random.Random(77)
    n = 0
    for _ in range(120):
        s = _random_table_constraints(rng) if rng.random() < 0.5 else _random_constraints(rng)
        root = And(*s)
        for m in _random_table_models(rng, 4, None):
            got = ModelRef(m).eval(root, model_completion=True)
            assert got.raw.op == "const", root
            assert got.raw.param == evaluate(root.raw, m), (s, m)
            n += got.raw.param
    assert n > 20


def test_eval_of_terms_and_partial_models():
    x, y = BVS("x", 256), BVS("y", 256)
    m = ModelRef({"x": 5})
    assert m.eval(x + BVV(1, 256)).value == 6
    part = m.eval(x + y)                      # y undeclared: stays symbolic
    assert part.symbolic and part.raw.op == "bvadd" and part.raw.args[0].op == "const"
    assert m.eval(x + y, model_completion=True).value == 5
    f = Function("keccak256_256", [256], 256)
    m2 = ModelRef({"x": 9, "keccak256_256": FuncInterp(3, {(9,): 42})})
    assert m2.eval(f(x)).value == 42
    assert m2.eval(f(BVV(1, 256))).value == 3
    assert m2.eval(f(y)).symbolic
    assert m2.eval(Not(f(x) == BVV(42, 256)), model_completion=True).raw.param == 0


def test_multi_model_lookup_order():
    x, y = BVS("x", 256), BVS("y", 256)
    a, b = ModelRef({"x": 1}), ModelRef({"y": 2, "x": 7})
    m = Model([a, b])
    assert m.decls() == ["x", "y", "x"]
    assert m["x"] == 1 and m["y"] == 2 and m["z"] is None
    assert m.eval(x).value == 1               # first model declaring x
    assert m.eval(y).value == 2
    # a conjunction's declaration (and) is declared by no model: the last one
    assert m.view(And(x == 7, y == 2)) is b
    assert m.eval(And(x == BVV(7, 256), y == BVV(2, 256)), model_completion=True).raw.param == 1
    assert _view(m, And(x == 7, y == 2).raw) == b.assignment
    assert _view(m, (x == 7).raw) == b.assignment
    assert Model({"x": 3}).eval(x).value == 3
    assert Model().eval(x) is None


def test_concrete_hash_data_from_model():
    km = KeccakFunctionManager()
    x = BVS("x", 256)
    km.create_keccak(x)
    km.create_keccak(BVS("q", 256))
    km.create_keccak(BVS("w", 512))
    model = Model([ModelRef({"x": 4, "keccak256_256": FuncInterp(0, {(4,): 99})})])
    assert km.get_concrete_hash_data(model) == {256: [99], 512: []}
