"""Pin the kernel-2 semantics (oracle/bv_ref.c, the program format kernel 2 runs)
on the reference's own SMT test data (tests/k2_pins.py): keccak_tests.py's
sat/unsat verdicts, the instruction tests' shift rows and EIP-145 tables as
programs, model_test.py's model surface.  CPU only: the oracle and the
Python evaluator; tests/test_gpu_k2_pinning.py runs the same cases on the device."""
import numpy as np
import pytest

from k2_pins import (adversarial_pool, keccak_cases, load, reference_interval_sequence,
                     shift_cases, witness, BVS, BVV)
from mythril_amd.smt.expr import And
from mythril_amd.smt.flatten import compile_sets
from mythril_amd.smt.keccak_manager import KeccakFunctionManager, TOTAL_PARTS
from mythril_amd.smt.program import ModelPool
from mythril_amd.smt.solver import Model, ModelCache
from oracle.bv_ref import eval_batch
from smt_eval import evaluate

NO = 0xFFFFFFFF


def test_fixture_shape():
    fx = load("keccak_cases.json")
    assert len(fx["basic"]) == 6 and len(fx["named"]) == 5
    assert [r["expected"] for r in fx["basic"]] == ["unsat", "unsat", "sat", "sat", "sat", "unsat"]


def test_interval_indices_follow_reference_order():
    """reset() keeps _index_counter (keccak_function_manager.py:48-54): the
    intervals of keccak_tests.py's cases, in its order, equal the reference's."""
    got = [c.intervals for c in keccak_cases()]
    assert got == reference_interval_sequence()


def test_reset_keeps_index_counter():
    km = KeccakFunctionManager()
    km.create_keccak(BVS("p", 256))
    c1 = km.create_conditions()
    i1 = km.interval_hook_for_size[256]
    km.reset()
    assert km.interval_hook_for_size == {} and km.concrete_hashes == {}
    km.create_keccak(BVS("p", 256))
    c2 = km.create_conditions()
    assert km.interval_hook_for_size[256] == i1 - 10 ** 30 == TOTAL_PARTS - 34534 - 10 ** 30
    assert c1.raw is not c2.raw                      # different bounds in the conjunct


def _compile(case):
    prog, kept = compile_sets([case.constraints])
    assert kept == [0], f"{case.name} does not compile for the device"
    return prog


def _pool(case, prog, models):
    return ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables)


@pytest.mark.parametrize("case", keccak_cases(), ids=lambda c: c.name)
def test_keccak_case_on_oracle(case):
    prog = _compile(case)
    root = And(*case.constraints).raw
    adv = adversarial_pool(case, 2048, seed=len(case.name))
    models = adv + ([witness(case)] if case.expected == "sat" else [])
    pool = _pool(case, prog, models)
    fs, sc = eval_batch(prog, pool)
    # the oracle equals the Python evaluation of the DAG as built (not lowered)
    py = [evaluate(root, m) for m in models[:512]] + ([evaluate(root, models[-1])]
                                                      if len(models) > 512 else [])
    first_py = next((k for k, v in enumerate(py[:512]) if v), None)
    if first_py is not None:
        assert fs[0] == first_py
    if case.expected == "sat":
        assert evaluate(root, models[-1]) == 1, "the witness must satisfy the axioms + query"
        one, _ = eval_batch(prog, _pool(case, prog, [models[-1]]))
        assert one[0] == 0
        assert sc[0] >= 1
    else:
        assert fs[0] == NO and sc[0] == 0, f"{case.name}: model {fs[0]} satisfies an unsat query"
        # near misses: a good share of the pool satisfies the keccak axioms themselves
        axioms_only, _ = compile_sets([[case.constraints[0]]])
        _, sc_ax = eval_batch(axioms_only, _pool(case, axioms_only, adv))
        assert sc_ax[0] > len(adv) // 20


@pytest.mark.parametrize("name,cons,model,truth", shift_cases(), ids=lambda x: x if isinstance(x, str) else "")
def test_shift_rows_on_oracle(name, cons, model, truth):
    prog, kept = compile_sets([[cons]])
    assert kept == [0]
    fs, sc = eval_batch(prog, ModelPool.from_dicts([model], prog.var_names, prog.var_widths))
    assert (sc[0] == 1) == truth
    assert evaluate(cons.raw, model) == int(truth)


from oracle_device import OracleK2 as _OracleEval  # noqa: E402  (kernel-2 stand-in, bv_ref)


def test_model_surface_on_quick_sat():
    """model_test.py:5-56: a model of x == 2 declares x, model[x] == 2 and
    model.eval(x) == 2 — here the model quick-sat returns from a cache of
    candidates, chosen by the kernel-2 program format (oracle)."""
    for case in load("model_cases.json"):
        x = BVS(case["var"]["name"], case["var"]["size"])
        expr = x == BVV(case["equals"]["value"], case["equals"]["size"])
        mc = ModelCache(device=_OracleEval())
        cands = [Model({x.raw.param: v}) for v in (5, 2, 0, 2 ** 255)]
        for m in cands:
            mc.put(m, 1)
        got = mc.check_quick_sat(expr.raw)
        assert got is cands[1]
        assert x.raw.param in got.decls()
        assert got[x.raw.param] == 2
        assert got.eval(x).value == 2 and got.eval(x.raw).param == 2
        if case["expected_value"] is not None:
            assert got.eval(x).value == case["expected_value"]
