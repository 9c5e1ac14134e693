"""Kernel-2 cases built from the reference's own SMT test data (tests/golden/*.json,
written by tests/golden/make_fixtures.py) — shared by the CPU pins
(test_k2_pinning.py: oracle/bv_ref.c + the Python evaluator) and the MI355X
parity test (test_gpu_k2_pinning.py).

* keccak_cases.json — tests/laser/keccak_tests.py:7-145.  Every test is restated
  on this repo's KeccakFunctionManager in the reference's file order with ONE
  manager (the reference's module-global `keccak_function_manager`), because
  reset() keeps `_index_counter` (keccak_function_manager.py:48-54) and the
  interval of a size first seen after a reset depends on the tests before it.
  The query of each test is create_conditions() ∧ (o1 == o2) [∧ extra], the
  conjunction the reference's Solver checks.  Expected sat/unsat comes from
  the fixture (z3's verdict in the reference's suite).  Kernel 2 can only ever
  answer SAT with a model: a sat case must be satisfied by the witness model
  built from the axioms below; an unsat case must be satisfied by no model of
  an adversarial pool whose models each satisfy most of the conjuncts.
* shift_rows.json / shift_vectors.json — tests/instructions/{shl,shr,sar}_test.py:
  `bvshl/bvlshr/bvashr(value, shift) == expected` as programs over variables,
  so the device shifts (the concrete values come from the model).
* model_cases.json — tests/laser/smt/model_test.py:5-56.
"""
from __future__ import annotations

import json
import random
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List

from mythril_amd.smt.expr import LShR, symbol_factory
from mythril_amd.smt.keccak_manager import (INTERVAL_DIFFERENCE, PART, TOTAL_PARTS,
                                            KeccakFunctionManager)
from mythril_amd.smt.program import FuncInterp
from smt_eval import evaluate

GOLDEN = Path(__file__).resolve().parent / "golden"
BVS, BVV = symbol_factory.BitVecSym, symbol_factory.BitVecVal
M256 = (1 << 256) - 1


def load(name):
    return json.loads((GOLDEN / name).read_text())


def bv(desc):
    if desc["kind"] == "val":
        return BVV(desc["value"], desc["size"])
    return BVS(desc["name"], desc["size"])


@dataclass
class KeccakCase:
    name: str
    constraints: list
    expected: str                       # "sat" / "unsat" (z3's verdict in the reference suite)
    intervals: Dict[int, int]           # input size -> interval index used by this case
    concrete: Dict[int, List[tuple]] = field(default_factory=dict)   # size -> [(input, hash)]
    symbolic: List = field(default_factory=list)                     # symbolic inputs, creation order
    var_names: List[str] = field(default_factory=list)
    targets: List[int] = field(default_factory=list)                 # constants the query compares to


def _case(km: KeccakFunctionManager, name, extra, expected, var_names, targets=()):
    cons = [km.create_conditions()] + list(extra)
    concrete: Dict[int, List[tuple]] = {}
    for c, h in km.concrete_hashes.items():
        concrete.setdefault(c.size(), []).append((c.value, h.value))
    symbolic = [x for xs in km.symbolic_inputs.values() for x in xs]
    tg = list(targets) + [h for v in concrete.values() for _, h in v]
    return KeccakCase(name, cons, expected, dict(km.interval_hook_for_size), concrete, symbolic,
                      list(var_names), tg)


def keccak_cases() -> List[KeccakCase]:
    fx = load("keccak_cases.json")
    km = KeccakFunctionManager()
    out: List[KeccakCase] = []
    for test in fx["order"]:
        if test == "test_keccak_basic":                       # keccak_tests.py:30-38
            for k, row in enumerate(fx["basic"]):
                km.reset()
                i1, i2 = bv(row["input1"]), bv(row["input2"])
                o1, o2 = km.create_keccak(i1), km.create_keccak(i2)
                names = [d["name"] for d in (row["input1"], row["input2"]) if d["kind"] == "sym"]
                out.append(_case(km, f"basic[{k}]", [o1 == o2], row["expected"], names))
            continue
        exp = fx["named"][test]
        km.reset()
        if test == "test_keccak_symbol_and_val":              # :41-56
            hundred, n = BVV(100, 256), BVS("n", 256)
            o1, o2 = km.create_keccak(hundred), km.create_keccak(n)
            out.append(_case(km, test, [o1 == o2, n == BVV(10, 256)], exp, ["n"], [10, 100]))
        elif test in ("test_keccak_complex_eq", "test_keccak_complex_eq2"):   # :59-107
            a, b = BVS("a", 160), BVS("b", 160)
            o1, o2 = km.create_keccak(a), km.create_keccak(b)
            two = BVV(2, 256)
            o1, o2 = km.create_keccak(two * o1), km.create_keccak(two * o2)
            extra = [o1 == o2] + ([a != b] if test == "test_keccak_complex_eq" else [])
            out.append(_case(km, test, extra, exp, ["a", "b"]))
        elif test == "test_keccak_simple_number":             # :110-124
            a = BVS("a", 160)
            o = km.create_keccak(a)
            out.append(_case(km, test, [BVV(10, 256) == o], exp, ["a"], [10]))
        elif test == "test_keccak_other_num":                 # :127-145
            a, b = BVS("a", 160), BVS("b", 256)
            o = km.create_keccak(BVV(2, 256) * km.create_keccak(a))
            out.append(_case(km, test, [b == o], exp, ["a", "b"]))
        else:
            raise AssertionError(f"keccak_cases.json names an unknown test {test}")
    return out


def reference_interval_sequence() -> List[Dict[int, int]]:
    """The interval indices the reference assigns, restated from
    keccak_function_manager.py:38-54,150-163 for keccak_tests.py's order: the
    counter starts at TOTAL_PARTS - 34534, is never reset, and drops by
    INTERVAL_DIFFERENCE each time create_conditions meets a size its (reset)
    interval table lacks — sizes in symbolic_inputs insertion order."""
    base = TOTAL_PARTS - 34534
    k = iter(range(100))
    nxt = lambda: base - next(k) * INTERVAL_DIFFERENCE          # noqa: E731
    seq = [{}, {}, {}, {256: nxt()}, {256: nxt()}, {256: nxt()},     # basic[0..5]
           {256: nxt()}]                                             # symbol_and_val
    for _ in range(2):                                               # complex_eq, complex_eq2
        a160 = nxt()
        seq.append({160: a160, 256: nxt()})
    seq.append({160: nxt()})                                         # simple_number
    a160 = nxt()
    seq.append({160: a160, 256: nxt()})                              # other_num
    return seq


# ------------------------------------------------------------------ models
def _interval(case: KeccakCase, size: int):
    lo = case.intervals[size] * PART
    return lo, lo + PART


def build_model(case: KeccakCase, assign: Dict[str, int], rng: random.Random = None) -> dict:
    """A model over the case's variables and keccak functions.  Without rng it is
    the witness the axioms admit: f_N(c) = keccak(c) for concrete inputs, each
    distinct symbolic input value gets the next 64-aligned value of its size's
    interval (or the concrete hash of an equal concrete input), inverses map
    back.  With rng every choice may be perturbed (adversarial pool)."""
    m: Dict[str, object] = dict(assign)
    funcs: Dict[int, Dict[tuple, int]] = {}
    invs: Dict[int, Dict[tuple, int]] = {}
    for size, pairs in case.concrete.items():
        for c, h in pairs:
            funcs.setdefault(size, {})[(c,)] = h
            invs.setdefault(size, {})[(h,)] = c
    fresh: Dict[int, int] = {}

    def publish():
        for size in set(funcs) | set(invs):
            m[f"keccak256_{size}"] = FuncInterp(0, funcs.get(size, {}))
            m[f"keccak256_{size}-1"] = FuncInterp(0, invs.get(size, {}))

    for x in case.symbolic:
        publish()
        size = x.size()
        v = evaluate(x.raw, m)
        f = funcs.setdefault(size, {})
        if (v,) in f and (rng is None or rng.random() < 0.8):
            continue
        lo, hi = _interval(case, size)
        j = fresh.get(size, 0)
        fresh[size] = j + 1
        h = ((lo + 63) // 64) * 64 + 64 * j
        inv_v = v
        if rng is not None:
            r = rng.random()
            if r < 0.25 and case.targets:
                h = rng.choice(case.targets)
            elif r < 0.35:
                h = rng.choice([lo - 64, hi, ((hi - 1) // 64) * 64, lo + 1])
            elif r < 0.45:
                h = rng.getrandbits(256)
            elif r < 0.55:
                others = [hh for s, ps in case.concrete.items() for _, hh in ps]
                h = rng.choice(others) if others else h
            if rng.random() < 0.1:
                inv_v = v ^ 1
        f[(v,)] = h & M256
        invs.setdefault(size, {})[(h & M256,)] = inv_v & ((1 << size) - 1)
    publish()
    return m


def witness(case: KeccakCase) -> dict:
    """Variable choices that make the sat cases true: equal symbolic inputs
    where the query equates two hashes; the concrete input where it equates a
    symbolic hash with a concrete one."""
    if case.name == "basic[4]":
        return build_model(case, {"N1": 100})
    assign = {n: 7 for n in case.var_names}
    m = build_model(case, assign)
    if case.name == "test_keccak_other_num":
        outer = case.symbolic[-1]           # b == keccak256_256(2 * keccak256_160(a))
        m["b"] = m[f"keccak256_{outer.size()}"].entries[(evaluate(outer.raw, m),)]
    return m


def adversarial_pool(case: KeccakCase, n: int, seed: int) -> List[dict]:
    rng = random.Random(seed)
    specials = [0, 1, 7, 10, 100, 2 ** 159, (1 << 160) - 1]
    out = []
    for _ in range(n):
        assign = {}
        shared = rng.choice(specials + [rng.getrandbits(160)])
        for name in case.var_names:
            r = rng.random()
            assign[name] = shared if r < 0.5 else rng.choice(specials + [rng.getrandbits(256)])
        m = build_model(case, assign, rng)
        if "b" in case.var_names and rng.random() < 0.5 and case.symbolic:
            try:                                # b equal to the outer hash (other_num shape)
                m["b"] = m[f"keccak256_{case.symbolic[-1].size()}"].entries[
                    (evaluate(case.symbolic[-1].raw, m),)]
            except KeyError:
                pass
        out.append(m)
    return out


# ------------------------------------------------------------------ shifts
def shift_cases():
    """(name, constraint, model dict, expected truth) for every reference shift
    row: value and shift are variables of the model, so the device shifts."""
    rows = load("shift_rows.json")
    vec = load("shift_vectors.json")
    v, s = BVS("value", 256), BVS("shift", 256)
    ops = {"shl": lambda a, b: a << b, "shr": LShR, "sar": lambda a, b: a >> b}
    out = []
    for op, f in ops.items():
        for k, r in enumerate(rows[op]):
            exp = r["expected"]["value"] & M256
            if r["value"]["kind"] == "sym":
                # a << 270 == 0 for every a (shl_test.py:33): several values of a
                for j, a in enumerate([0, 1, M256, 0xDEADBEEF << 100]):
                    out.append((f"{op}_row{k}_a{j}", f(v, s) == BVV(exp, 256),
                                {"value": a, "shift": r["shift"]["value"] & M256}, True))
                continue
            val, sh = r["value"]["value"] & M256, r["shift"]["value"] & M256
            out.append((f"{op}_row{k}", f(v, s) == BVV(exp, 256), {"value": val, "shift": sh}, True))
            out.append((f"{op}_row{k}_neg", f(v, s) == BVV(exp ^ 1, 256),
                        {"value": val, "shift": sh}, False))
        for k, r in enumerate(vec[op]):
            val, sh, exp = (int(r[x], 16) for x in ("value", "shift", "expected"))
            out.append((f"{op}_eip145_{k}", f(v, s) == BVV(exp, 256), {"value": val, "shift": sh}, True))
            out.append((f"{op}_eip145_{k}_neg", f(v, s) == BVV(exp ^ (1 << 255), 256),
                        {"value": val, "shift": sh}, False))
    return out
