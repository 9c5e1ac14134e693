"""Kernel-2 host layer on CPU: expression layer, flattener, C4 generator and the
oracle evaluator agree with a pure-Python evaluation of the expressions."""
import random

import numpy as np
import pytest

from mythril_amd.smt import synth
from mythril_amd.smt.expr import (And, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow,
                                  Concat, Extract, If, Not, Or, SignExt, UDiv, UGE, UGT, ULE,
                                  ULT, URem, SRem, LShR, ZeroExt, symbol_factory, Node)
from mythril_amd.smt.flatten import Compiler, Unsupported, compile_sets
from mythril_amd.smt.program import ModelPool
from oracle.bv_ref import eval_batch
from smt_eval import evaluate

BVS, BVV = symbol_factory.BitVecSym, symbol_factory.BitVecVal


def test_c4_programs_match_expressions():
    dr = synth.Draws(300, seed=synth.C4_SEED)
    prog = synth.c4_programs(dr)
    models = synth.c4_models(96)
    fs, sc = eval_batch(prog, models)
    for i in range(0, 300, 3):
        e = synth.dag_expr(dr, i)
        vals = [evaluate(e, synth.model_dict(models, m)) for m in range(96)]
        first = next((m for m, v in enumerate(vals) if v), 0xFFFFFFFF)
        assert (first, sum(vals)) == (fs[i], sc[i]), i


def test_c4_full_size_shape_and_determinism():
    dr = synth.Draws(1000, seed=synth.C4_SEED)
    a = synth.c4_programs(dr)
    b = synth.c4_programs(synth.Draws(1000, seed=synth.C4_SEED))
    assert np.array_equal(a.insns, b.insns) and np.array_equal(a.prog_off, b.prog_off)
    lens = np.diff(a.prog_off.astype(np.int64))
    # a level an ite(spine == leaf, spine, leaf) discards emits nothing, so a DAG
    # can shrink to its root compare
    assert 1 <= lens.min() and lens.max() <= 2 + 3 * synth.LEVELS
    assert 28 < lens.mean() < 40          # ~65 nodes per DAG, about 34 instructions


def test_c4_programs_have_the_compilers_form():
    """The generator emits what flatten.Compiler emits for the same DAG (no
    copies, select-of-compare folded, zero-extension aliased, dead levels
    dropped): per DAG the same multiset of opcodes, except that the compiler
    also shares a repeated extract of the same leaf across levels (CSE through
    an extra slot; the generator keeps to two slots), and a min/max of a value
    with itself may fold either way."""
    from collections import Counter
    from mythril_amd.smt.program import OPS
    norm = {"bvumax": "bvumin", "bvsmax": "bvsmin"}
    # operand-swapped forms (flatten._SWAPPED: the accumulator is only operand A)
    canon = {"rconcat": "concat", "bvrsub": "bvsub", "bvugt": "bvult", "bvuge": "bvule",
             "bvsgt": "bvslt", "bvsge": "bvsle"}
    dr = synth.Draws(300, seed=synth.C4_SEED + 5)
    prog = synth.c4_programs(dr)
    n = exact = 0
    for i in range(300):
        try:
            p = Compiler().compile(synth.dag_expr(dr, i))
        except Unsupported:
            continue
        a = Counter(canon.get(OPS[int(w) & 0xFF], OPS[int(w) & 0xFF]) for w in p[:, 0])
        b = Counter(canon.get(OPS[int(w) & 0xFF], OPS[int(w) & 0xFF]) for w in prog.program(i)[:, 0])
        exact += a == b
        extra = b - a
        assert not (a - b) - Counter({k: v for k, v in (a - b).items() if k in norm or k in norm.values()}), i
        assert set(extra) <= {"extract"} | set(norm) | set(norm.values()), (i, extra)
        n += 1
    assert n > 250 and exact > 0.9 * n


def _random_constraints(rng, n_terms=6):
    x, y, z = BVS("x", 256), BVS("y", 256), BVS("z", 256)
    cd = BVS("cd4", 8)
    terms = [x + y, x - z, x * y, UDiv(x, y), URem(z, x), x / y, SRem(y, z), x & z, x | y,
             x ^ y, ~x, LShR(x, BVV(7, 256)), x << BVV(3, 256), x >> BVV(200, 256),
             If(ULT(x, y), x, z), Concat(Extract(127, 0, x), Extract(127, 0, y)),
             ZeroExt(248, cd), SignExt(248, cd), Extract(7, 0, x + z)]
    preds = []
    for _ in range(n_terms):
        a, b = rng.choice(terms), rng.choice(terms)
        if a.size() != b.size():
            b = Extract(a.size() - 1, 0, ZeroExt(256 - b.size(), b)) if b.size() < 256 else \
                Extract(a.size() - 1, 0, b)
        k = rng.randrange(12)
        preds.append([ULT(a, b), UGT(a, b), ULE(a, b), UGE(a, b), a < b, a > b, a <= b, a >= b,
                      a == b, a != b,
                      BVAddNoOverflow(a, b, False) if a.size() == b.size() else a == b,
                      BVSubNoUnderflow(a, b, False)][k])
    if rng.random() < 0.5:
        preds.append(Or(preds[0], Not(preds[-1])))
    if rng.random() < 0.3:
        preds.append(BVMulNoOverflow(x, y, False))
    return preds


def test_flattener_matches_python_semantics():
    rng = random.Random(1234)
    sets = [_random_constraints(rng, rng.randrange(1, 8)) for _ in range(120)]
    prog, kept = compile_sets(sets)
    assert len(kept) == len(sets)
    models_py = []
    mrng = random.Random(99)
    specials = [0, 1, 2, (1 << 255), (1 << 256) - 1, (1 << 160) - 1]
    for _ in range(64):
        models_py.append({name: (mrng.choice(specials) if mrng.random() < 0.3 else
                                 mrng.getrandbits(w)) & ((1 << w) - 1)
                          for name, w in zip(prog.var_names, prog.var_widths)})
    pool = ModelPool.from_dicts(models_py, prog.var_names, prog.var_widths)
    fs, sc = eval_batch(prog, pool)
    for d, s in enumerate(sets):
        root = And(*s)
        vals = [evaluate(root.raw, m) for m in models_py]
        first = next((m for m, v in enumerate(vals) if v), 0xFFFFFFFF)
        assert (first, sum(vals)) == (fs[d], sc[d]), d


def test_flattener_slot_pressure_and_unsupported():
    x = BVS("x", 256)
    # 40 conjuncts fold one by one: only the running result needs a slot
    many = [ULT(x + BVV(k, 256), BVV(10 ** 6 + k, 256)) for k in range(40)]
    prog, kept = compile_sets([many])
    assert kept == [0] and prog.n_slots <= 2
    wide = Concat(x, x)                   # 512-bit keccak-style input: split in two chunks
    prog2, kept2 = compile_sets([[wide == Concat(x, BVV(3, 256))]])
    assert kept2 == [0]
    wider = Concat(x, x, x)               # 768-bit equality: three chunk compares
    prog3, kept3 = compile_sets([[wider == Concat(x, x, BVV(1, 256))]])
    assert kept3 == [0]
    prog4, kept4 = compile_sets([[wide + wide == wide]])    # 512-bit arithmetic: z3
    assert kept4 == []


def test_constant_folding_follows_z3():
    assert (UDiv(BVV(5, 256), BVV(0, 256))).value == (1 << 256) - 1
    assert (URem(BVV(5, 256), BVV(0, 256))).value == 5
    assert (BVV(-7, 256) / BVV(2, 256)).value == (-3) % (1 << 256)
    assert (BVV(1, 256) < BVV(-1, 256)).value is False     # signed <, bitvec.py:140-150
    assert ULE(BVV(3, 256), BVV(3, 256)).value is True


# ------------------------------------------------ arrays, functions, keccak conjuncts
from mythril_amd.smt.expr import Array, Function, K  # noqa: E402
from mythril_amd.smt.program import ArrayInterp, FuncInterp  # noqa: E402

M256 = (1 << 256) - 1


def _random_table_constraints(rng):
    """Constraint sets of the shapes LASER builds: storage
    arrays with symbolic and concrete stores, calldata byte arrays, keccak
    functions of 256- and 512-bit inputs with the inverse and interval conjuncts
    of keccak_function_manager.py:150-179, Power."""
    x, y, s = BVS("x", 256), BVS("y", 256), BVS("slot", 256)
    storage = Array("Storage", 256, 256)
    if rng.random() < 0.7:
        storage[x] = y
    if rng.random() < 0.5:
        storage[BVV(1, 256)] = x + y
    if rng.random() < 0.3:
        storage[y] = BVV(rng.getrandbits(8), 256)
    cd = K(256, 8, 0) if rng.random() < 0.5 else Array("calldata", 256, 8)
    for k in range(rng.randrange(0, 4)):
        cd[BVV(k, 256)] = Extract(7, 0, x >> BVV(8 * k, 256))
    f512 = Function("keccak256_512", [512], 256)
    inv512 = Function("keccak256_512-1", [256], 512)
    f256 = Function("keccak256_256", [256], 256)
    power = Function("Power", [256, 256], 256)
    key = Concat(x, s)
    h = f512(key)
    lo = BVV(rng.getrandbits(255), 256)
    pool = [
        storage[x] == y, ULT(storage[s], BVV(1 << 200, 256)), storage[BVV(1, 256)] != BVV(0, 256),
        Concat(cd[BVV(0, 256)], cd[BVV(1, 256)]) == Extract(15, 0, x),
        ZeroExt(248, cd[y]) == BVV(0, 256),
        inv512(h) == key, ULE(lo, h), ULT(h, lo + BVV(1 << 120, 256)),
        URem(h, BVV(64, 256)) == BVV(0, 256),
        f512(Concat(BVV(0xDEAD, 256), BVV(0, 256))) == BVV(rng.getrandbits(256), 256),
        f256(y) == x, Extract(255, 0, inv512(f256(x))) == x,
        power(BVV(2, 256), y) == x, storage[h] == BVV(0, 256),
        Or(f512(key) == BVV(5, 256), And(key == Concat(y, BVV(0, 256)), f256(x) != y)),
    ]
    return [rng.choice(pool) for _ in range(rng.randrange(1, 6))]


def _random_table_models(rng, n, prog):
    """Models whose interpretations often contain the keys the constraints touch."""
    out = []
    for _ in range(n):
        x, y, s = rng.getrandbits(256), rng.getrandbits(256), rng.choice([0, 1, 2, rng.getrandbits(256)])
        if rng.random() < 0.3:
            y = x
        m = {"x": x, "y": y, "slot": s}
        h = rng.getrandbits(256) & ~63 if rng.random() < 0.7 else rng.getrandbits(256)
        if rng.random() < 0.8:
            m["Storage"] = ArrayInterp(rng.choice([0, 7]), {x: rng.choice([y, 0]), 1: rng.getrandbits(8),
                                                            s: rng.getrandbits(201)})
        if rng.random() < 0.5:
            m["calldata"] = ArrayInterp(0, {y: 0, 0: x & 0xFF})
        if rng.random() < 0.8:
            m["keccak256_512"] = FuncInterp(rng.choice([0, 5]), {((x << 256) | s,): h,
                                                                   ((y << 256),): 5})
        if rng.random() < 0.7:
            m["keccak256_512-1"] = FuncInterp(0, {(h,): (x << 256) | s})
        if rng.random() < 0.7:
            m["keccak256_256"] = FuncInterp(rng.getrandbits(256), {(y,): x, (x,): rng.getrandbits(256)})
        if rng.random() < 0.5:
            m["Power"] = FuncInterp(1, {(2, y): x})
        out.append(m)
    return out


def test_arrays_functions_wide_values_match_python_semantics():
    rng = random.Random(4321)
    sets = [_random_table_constraints(rng) for _ in range(150)]
    prog, kept = compile_sets(sets)
    assert len(kept) == len(sets)
    assert {t.name for t in prog.tables} >= {"Storage", "keccak256_512", "keccak256_512-1"}
    models = _random_table_models(random.Random(8), 80, prog)
    pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables)
    fs, sc = eval_batch(prog, pool)
    hits = 0
    for d, s in enumerate(sets):
        root = And(*s)
        vals = [evaluate(root.raw, m) for m in models]
        first = next((m for m, v in enumerate(vals) if v), 0xFFFFFFFF)
        assert (first, sum(vals)) == (fs[d], sc[d]), (d, s)
        hits += sum(vals)
    assert hits > 100            # the generator reaches satisfying interpretations


def test_select_store_folding_follows_z3_simplify():
    x = BVS("x", 256)
    st = K(256, 256, 0)
    st[BVV(1, 256)] = BVV(5, 256)
    assert st[BVV(1, 256)].value == 5 and st[BVV(2, 256)].value == 0
    a = Array("S", 256, 256)
    a[BVV(1, 256)] = x
    assert a[BVV(1, 256)].raw is x.raw
    # a store at a different constant index is skipped: select(S, 2)
    assert a[BVV(2, 256)].raw.args[0].op == "array"


def test_accumulator_is_only_operand_a():
    """bv_eval.cuh loads operand A into the accumulator's registers, so the
    compiler never leaves the accumulator in operand B or C: it swaps
    commutative ops, reverses compares, uses bvrsub / rconcat, or spills to a
    slot (flatten._acc_ok).  Checked on random sets and on the C4 generator."""
    from mythril_amd.smt.program import OPCODE, REF_ACC
    rng = random.Random(99)
    sets = [_random_constraints(rng, rng.randrange(1, 10)) for _ in range(300)]
    prog, kept = compile_sets(sets)
    assert len(kept) > 250
    ops = prog.insns[:, 0] & 0xFF
    unary = {OPCODE[o] for o in ("copy", "bvnot", "bvneg", "not", "extract", "zero_extend", "sign_extend")}
    for w, op in zip(prog.insns, ops):
        nref = 3 if op == OPCODE["ite"] else (1 if op in unary else 2)
        assert all(int(w[1 + k]) >> 30 != REF_ACC for k in range(1, nref))
    assert (ops == OPCODE["bvrsub"]).any() or (ops == OPCODE["bvugt"]).any()
    c4 = synth.c4_programs(synth.Draws(2000, seed=synth.C4_SEED))
    ops4 = c4.insns[:, 0] & 0xFF
    for w, op in zip(c4.insns, ops4):
        nref = 3 if op == OPCODE["ite"] else (1 if op in unary else 2)
        assert all(int(w[1 + k]) >> 30 != REF_ACC for k in range(1, nref))


def test_programs_with_more_than_eight_live_values():
    """The flattener allows 16 slots (kernel 2's 4-bit slot field): a set that
    keeps 10 values live compiles, and the oracle evaluator agrees with the
    pure-Python DAG evaluation on it."""
    import random as _r
    from mythril_amd.smt.expr import Array, UGT, symbol_factory
    from mythril_amd.smt.program import ArrayInterp, ModelPool
    from oracle.bv_ref import eval_batch
    from smt_eval import evaluate
    BVS = symbol_factory.BitVecSym
    xs = [BVS(f"x{k}", 256) for k in range(24)]

    def tree(lo, hi):
        if hi - lo == 1:
            return xs[lo] * xs[(lo + 7) % 24]
        mid = (lo + hi) // 2
        return tree(lo, mid) + tree(mid, hi)
    bal = Array("balance", 256, 256)
    for k in range(6):
        bal[xs[k]] = bal[xs[k]] + xs[k + 6]
    sets = [[tree(0, 24) == xs[0]], [UGT(bal[xs[1]] + bal[xs[2]] * bal[xs[3]], bal[xs[4]] - bal[xs[5]])]]
    prog, kept = compile_sets(sets)
    assert kept == [0, 1] and 8 < prog.n_slots <= 16
    rng = _r.Random(16)
    models = []
    for m in range(60):
        a = {f"x{k}": rng.choice([0, 1, 2, rng.getrandbits(256), rng.getrandbits(8)]) for k in range(24)}
        a["balance"] = ArrayInterp(rng.getrandbits(64), {a["x1"]: rng.getrandbits(256)})
        models.append(a)
    pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables)
    fs, sc = eval_batch(prog, pool)
    for d, s_ in enumerate(sets):
        vals = [evaluate(s_[0].raw, m) for m in models]
        assert (next((i for i, v in enumerate(vals) if v), 0xFFFFFFFF), sum(vals)) == (fs[d], sc[d])


def test_native_compiler_programs_equal_the_python_passes():
    """mg_cc_* (csrc/cc.h) against flatten.PyCompiler: on C4 DAGs, random
    operator sets, array / function-table sets and >8-slot sets, both compilers
    accept the same sets, use as many instructions, and their programs give the
    same first-satisfying model and count on the oracle evaluator (instruction
    order may differ only where equal-size operand subtrees tie)."""
    from mythril_amd.smt.flatten import NativeCompiler, PyCompiler
    rng = random.Random(77)
    dr = synth.Draws(200, seed=synth.C4_SEED + 17)
    sets = [[synth.dag_expr(dr, i)] for i in range(200)]
    sets += [_random_constraints(rng) for _ in range(150)]
    sets += [_random_table_constraints(rng) for _ in range(150)]
    pn, kn = compile_sets(sets, NativeCompiler())
    pp, kp = compile_sets(sets, PyCompiler())
    assert kn == kp and len(kn) > 400
    assert np.array_equal(np.diff(pn.prog_off.astype(np.int64)), np.diff(pp.prog_off.astype(np.int64)))
    assert set(pn.var_names) == set(pp.var_names)
    models = _random_table_models(random.Random(5), 160, pp)
    out = []
    for prog in (pn, pp):
        pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables)
        out.append(eval_batch(prog, pool))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert 0 < int(out[1][1].sum()) < len(kn) * 160


def test_constant_index_selects_are_pool_variables():
    """select(Array, const) lowers to a model-pool variable (no table): its
    column reads the array interpretation's entry or default, and a
    PoolColumns column is rebuilt when the array's revision moves."""
    from mythril_amd.smt.lower import select_var
    from mythril_amd.smt.program import PoolColumns
    cd = Array("7_calldata", 256, 8)
    sets = [[cd[BVV(4, 256)] == BVV(0x2A, 8)], [ULT(ZeroExt(248, cd[BVV(0, 256)]), BVV(3, 256))]]
    prog, kept = compile_sets(sets)
    assert len(kept) == 2 and not prog.tables
    assert set(prog.var_names) == {select_var("7_calldata", 4), select_var("7_calldata", 0)}
    models = [{"7_calldata": ArrayInterp(0x2A, {0: 9})}, {"7_calldata": ArrayInterp(0, {4: 0x2A, 0: 2})},
              {"7_calldata": ArrayInterp(1, {})}, {}]
    want = [[evaluate(And(*s).raw, m) for m in models] for s in sets]
    fs, sc = eval_batch(prog, ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables))
    assert [sum(w) for w in want] == list(sc) == [2, 3]
    rev = [0]
    cols = PoolColumns(models, revision=lambda name: rev[0] if name == "7_calldata" else 0)
    assert (cols.pool(prog.var_names, prog.var_widths).values
            == ModelPool.from_dicts(models, prog.var_names, prog.var_widths).values).all()
    models[3]["7_calldata"] = ArrayInterp(0x2A, {})
    rev[0] += 1
    _, sc2 = eval_batch(prog, cols.pool(prog.var_names, prog.var_widths, prog.tables))
    assert list(sc2) == [3, 2]


def test_dense_array_interpretations_read_like_entry_dicts():
    """A witness seed's calldata is held as bytes (ArrayInterp dense=) until
    something takes its entry dict: pools built from either form agree."""
    from mythril_amd.smt.program import PoolColumns
    cd = Array("3_calldata", 256, 8)
    sets = [[cd[BVV(k, 256)] == BVV(k + 1, 8)] for k in (0, 2, 5, 70)] + \
           [[cd[BVS("i", 256)] == BVV(3, 8)]]
    prog, kept = compile_sets(sets)
    assert len(kept) == len(sets)
    data = [bytes([1, 9, 3, 4, 5, 6]), bytes([1, 2, 3]), b"", bytes(range(1, 80))]
    dense = [{"3_calldata": ArrayInterp(d, dense=x), "i": 2} for d, x in zip((0, 6, 0, 1), data)]
    plain = [{"3_calldata": ArrayInterp(d, dict(enumerate(x))), "i": 2} for d, x in zip((0, 6, 0, 1), data)]
    a = PoolColumns(dense).pool(prog.var_names, prog.var_widths, prog.tables)
    b = PoolColumns(plain).pool(prog.var_names, prog.var_widths, prog.tables)
    assert (a.values == b.values).all()
    assert [list(x) for x in eval_batch(prog, a)] == [list(x) for x in eval_batch(prog, b)]
    want = [sum(evaluate(And(*s).raw, m) for m in plain) for s in sets]
    assert list(eval_batch(prog, a)[1]) == want
    assert dense[0]["3_calldata"].untouched_dense() is not None
    dense[0]["3_calldata"].entries[0] = 7          # taken and changed: the dict is what counts
    assert dense[0]["3_calldata"].untouched_dense() is None
    assert PoolColumns(dense).pool(prog.var_names, prog.var_widths).values[prog.var_names.index(
        "3_calldata\x1f0"), 0, 0] == 7
