"""Kernel 2 parity on an MI355X: device first-satisfying-model and satisfying counts
equal the CPU oracle (oracle/bv_ref.c) bit-exactly."""
import random

import numpy as np
import pytest

from mythril_amd.device import GpuDevice
from mythril_amd.smt import synth
from mythril_amd.smt.flatten import compile_sets
from mythril_amd.smt.program import ModelPool
from oracle.bv_ref import eval_batch
from test_smt_programs import _random_constraints

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


@pytest.mark.parametrize("n_models", [1, 63, 256, 300, 1024])
def test_c4_small_device_equals_oracle(dev, n_models):
    prog = synth.c4_programs(synth.Draws(1500, seed=synth.C4_SEED + n_models))
    models = synth.c4_models(n_models, seed=5 + n_models)
    fs, sc, _ = dev.eval(prog, models)
    rfs, rsc = eval_batch(prog, models)
    assert np.array_equal(fs, rfs)
    assert np.array_equal(sc, rsc)


def test_flattened_constraint_sets_device_equals_oracle(dev):
    rng = random.Random(77)
    sets = [_random_constraints(rng, rng.randrange(1, 10)) for _ in range(400)]
    prog, kept = compile_sets(sets)
    mr = random.Random(5)
    specials = [0, 1, (1 << 255), (1 << 256) - 1]
    models = [{n: (mr.choice(specials) if mr.random() < 0.3 else mr.getrandbits(w)) & ((1 << w) - 1)
               for n, w in zip(prog.var_names, prog.var_widths)} for _ in range(512)]
    pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths)
    fs, sc, _ = dev.eval(prog, pool)
    rfs, rsc = eval_batch(prog, pool)
    assert np.array_equal(fs, rfs) and np.array_equal(sc, rsc)


def test_c4_full_size_sampled_parity(dev):
    """1M DAGs x 4096 models on the device; a random sample of DAGs re-evaluated by
    the oracle over all 4096 models; plus size-independent properties."""
    prog, models = synth.c4_batch(1_000_000, 4096)
    dev.eval_upload(prog, models)
    ms = dev.eval_run()
    fs, sc = dev.eval_download()
    assert ms > 0
    sat = sc > 0
    assert np.array_equal(sat, fs != 0xFFFFFFFF)
    assert (fs[sat] < 4096).all() and (sc <= 4096).all()
    rng = np.random.default_rng(3)
    sample = np.sort(rng.choice(prog.n_dags, 256, replace=False))
    for d in sample:
        rfs, rsc = eval_batch(prog, models, first=int(d), count=1, threads=1)
        assert (fs[d], sc[d]) == (rfs[0], rsc[0]), d
    # split runs over DAG ranges equal the whole
    dev.eval_run(0, 1000)
    a, b = dev.eval_download(0, 1000)
    assert np.array_equal(a, fs[:1000]) and np.array_equal(b, sc[:1000])


def test_arrays_functions_device_equals_oracle(dev):
    """Storage / calldata arrays, keccak256_N functions and their inverses, Power,
    512-bit keys (kernel-2 table lookups, BV_TAB) — device vs oracle."""
    from test_smt_programs import _random_table_constraints, _random_table_models
    rng = random.Random(2024)
    sets = [_random_table_constraints(rng) for _ in range(600)]
    prog, kept = compile_sets(sets)
    assert len(kept) == len(sets) and prog.tables
    models = _random_table_models(random.Random(11), 700, prog)
    pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables)
    fs, sc, _ = dev.eval(prog, pool)
    rfs, rsc = eval_batch(prog, pool)
    assert np.array_equal(fs, rfs) and np.array_equal(sc, rsc)
    assert (sc > 0).sum() > 50
    # a pool without tables after one with them (table state reset on upload)
    prog2, _ = compile_sets([[s for s in sets[0] if False] or [ULT_x()]])
    pool2 = ModelPool.from_dicts([{"x": 1}, {"x": 5}], prog2.var_names, prog2.var_widths)
    fs2, sc2, _ = dev.eval(prog2, pool2)
    assert list(fs2) == [0] and list(sc2) == [1]


def ULT_x():
    from mythril_amd.smt.expr import ULT, symbol_factory
    return ULT(symbol_factory.BitVecSym("x", 256), symbol_factory.BitVecVal(3, 256))


def test_plain_ops_and_tables_equal_oracle(dev):
    """The shipped kernel (scalar-load instruction fetch) on C4-mix programs and on
    array / function-table sets equals the oracle (333 and 300 models: partial
    model chunks)."""
    from test_smt_programs import _random_table_constraints, _random_table_models
    prog = synth.c4_programs(synth.Draws(900, seed=synth.C4_SEED + 9))
    models = synth.c4_models(333, seed=19)
    fs, sc, _ = dev.eval(prog, models)
    rfs, rsc = eval_batch(prog, models)
    assert np.array_equal(fs, rfs) and np.array_equal(sc, rsc)
    rng = random.Random(31)
    prog, _ = compile_sets([_random_table_constraints(rng) for _ in range(200)])
    pool = ModelPool.from_dicts(_random_table_models(random.Random(3), 300, prog), prog.var_names,
                                prog.var_widths, prog.tables)
    fs, sc, _ = dev.eval(prog, pool)
    rfs, rsc = eval_batch(prog, pool)
    assert np.array_equal(fs, rfs) and np.array_equal(sc, rsc)


def test_sixteen_slot_programs_equal_oracle(dev):
    """Programs that keep up to 16 values live (128 KiB of LDS per block): a
    balanced sum tree of distinct variable products needs a slot per pending
    subtree, and a path's balance store chain read at several keys."""
    from mythril_amd.smt.expr import Array, UGT, symbol_factory
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
    assert kept == [0, 1] and prog.n_slots > 8
    rng = random.Random(16)
    from mythril_amd.smt.program import ArrayInterp
    models = []
    for m in range(700):
        a = {f"x{k}": rng.choice([0, 1, 2, rng.getrandbits(256), rng.getrandbits(8)]) for k in range(24)}
        a["balance"] = ArrayInterp(rng.getrandbits(64), {a["x1"]: rng.getrandbits(256)})
        models.append(a)
    pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables)
    fs, sc, _ = dev.eval(prog, pool)
    rfs, rsc = eval_batch(prog, pool)
    assert np.array_equal(fs, rfs) and np.array_equal(sc, rsc)


@pytest.mark.parametrize("w", [8, 64, 255, 256])
def test_division_class_ops_at_every_width(dev, w):
    """UDIV UREM SDIV SREM SMOD and the unsigned multiply-overflow test share one
    division site in the kernel (bv_divop): each op at width w, against values
    at the sign / zero / all-ones edges (z3 zero-divisor semantics)."""
    from mythril_amd.smt.expr import (BVMulNoOverflow, SDiv, SMod, SRem, UDiv, URem,
                                      symbol_factory)
    BVS = symbol_factory.BitVecSym
    x, y, z = BVS("x", w), BVS("y", w), BVS("z", w)
    sets = []
    for f in (UDiv, URem, SDiv, SRem, SMod):
        sets.append([f(x, y) == z])
        sets.append([f(y, x) == z])
    sets.append([BVMulNoOverflow(x, y, False)])
    sets.append([BVMulNoOverflow(y, z, False)])
    prog, kept = compile_sets(sets)
    assert len(kept) == len(sets)
    m = (1 << w) - 1
    edges = [0, 1, 2, 3, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1, (1 << (w - 1)) + 1]
    rng = random.Random(w)
    from mythril_amd.smt import semantics
    models = []
    for k in range(1024):
        a = rng.choice(edges) if k % 3 else rng.getrandbits(w)
        b = rng.choice(edges) if k % 2 else rng.getrandbits(rng.choice([1, 5, w // 2 + 1, w]))
        op = ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")[k % 5]
        # every 4th model makes the first constraint of op k % 5 true
        c = semantics.apply_op(op, w, [a, b], [w, w], None) if k % 4 == 0 else rng.getrandbits(w)
        models.append({"x": a, "y": b, "z": c & m})
    pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths)
    fs, sc, _ = dev.eval(prog, pool)
    rfs, rsc = eval_batch(prog, pool)
    assert np.array_equal(fs, rfs) and np.array_equal(sc, rsc)
    assert (sc[:10] > 0).all()


def _fusable_programs(n_dags, seed):
    """Random programs made of the two fused shapes (bv_fuse in bv_eval.cuh):
    comparison -> Boolean and, and extract -> rconcat, with every comparison kind,
    signed widths 1..256, accumulator and slot operands, stored and unstored
    intermediates (a stored first instruction must stay unfused)."""
    from mythril_amd.smt.program import ProgramBatch
    O = synth.OPCODE
    rng = random.Random(seed)
    cmps = ["eq", "distinct", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge"]
    widths = [256, 64, 8]
    var = lambda i: (2 << 30) | i
    slot = lambda i: (1 << 30) | i
    const = lambda i: (3 << 30) | i

    def w0(op, width, store=None):
        return O[op] | (width << 8) | ((1 << 17) | (store << 18) if store is not None else 0)

    insns, off = [], [0]
    for _ in range(n_dags):
        prog = [[w0("copy", 256, 0), var(rng.randrange(3)), 0, 0]]          # slot 0: a variable
        prog.append([w0("extract", 1, 1), var(rng.randrange(3)), rng.randrange(256), 0])  # slot 1: a bit
        for _ in range(rng.randrange(2, 6)):
            if rng.random() < 0.3:
                # a chain of 256-bit binary ops over variables, constants and slot 0
                simple = ["bvadd", "bvsub", "bvmul", "bvand", "bvor", "bvxor", "bvumax", "bvumin", "bvrsub"]
                # (led half the time by another 256-bit op: the fused-tail shape)
                heads = ["bvnot", "bvshl", "bvlshr", "bvashr", "bvsmin", "bvsmax", "bvudiv", "bvurem", "bvsdiv"]
                for k in range(rng.randrange(2, 6)):
                    a = var(rng.randrange(3)) if k == 0 else 0
                    op = rng.choice(heads) if k == 0 and rng.random() < 0.5 else rng.choice(simple)
                    if k == 0 and rng.random() < 0.2:      # a narrower head: a 128-bit extract
                        prog.append([w0("extract", 128), a, rng.randrange(129), 0])
                        continue
                    prog.append([w0(op, 256, 0 if rng.random() < 0.15 else None), a,
                                 rng.choice([var(rng.randrange(3)), const(rng.randrange(2)), slot(0)]), 0])
            elif rng.random() < 0.6:
                # two sw-bit operands (slot 2 and the accumulator), compared, and-ed with slot 1
                k = rng.choice(cmps)
                sw = rng.choice([1, 7, 8, 64, 128, 255, 256])
                prog.append([w0("extract", sw, 2), var(rng.randrange(3)), rng.randrange(257 - sw), 0])
                prog.append([w0("extract", sw), var(rng.randrange(3)), rng.randrange(257 - sw), 0])
                prog.append([w0(k, 1, 2 if rng.random() < 0.2 else None), 0, slot(2), sw])
                prog.append([w0("and", 1, 1 if rng.random() < 0.5 else None), 0, slot(1), 0])
            else:
                # an hw-bit high part in slot 3, an ew-bit extract, rconcat'ed
                ew = rng.choice([1, 8, 100, 128, 255])
                hw = rng.choice([1, 8, 128, 256 - ew]) if ew < 256 else 0
                hw = max(1, min(hw, 256 - ew))
                prog.append([w0("extract", hw, 3), var(rng.randrange(3)), rng.randrange(257 - hw), 0])
                prog.append([w0("extract", ew, 2 if rng.random() < 0.2 else None), var(rng.randrange(3)),
                             rng.randrange(257 - ew), 0])
                prog.append([w0("rconcat", ew + hw, 0 if rng.random() < 0.5 else None), 0, slot(3), ew])
            prog.append([w0("and", 1), slot(1), slot(1), 0] if rng.random() < 0.3 else
                        [w0("bvugt", 1), slot(0), var(0), 256])
        insns += prog
        off.append(len(insns))
    consts = np.zeros((2, 8), dtype=np.uint32)
    consts[1, :] = 0xFFFFFFFF
    consts[1, 7] = 0x7FFFFFFF
    return ProgramBatch(np.asarray(insns, dtype=np.uint32), np.asarray(off, dtype=np.uint32), consts, 4,
                        ["x0", "x1", "x2"], [256, 256, 256])


def test_fused_programs_equal_unfused_and_oracle(dev, monkeypatch):
    """Superinstructions (MG_BV_FUSE, all shapes and chains by default): on programs
    dense in the fused shapes, and on C4's own, per-model bitmaps equal the unfused upload's and
    first/count equal the oracle, which always interprets the unfused program."""
    mr = random.Random(9)
    specials = [0, 1, (1 << 255), (1 << 256) - 1, (1 << 127), (1 << 63) - 1]
    models = [{n: mr.choice(specials) if mr.random() < 0.4 else mr.getrandbits(256) for n in ("x0", "x1", "x2")}
              for _ in range(320)]
    for prog, pool in ((_fusable_programs(600, 3), None),
                       (synth.c4_programs(synth.Draws(500, seed=synth.C4_SEED + 29)), synth.c4_models(300, seed=31))):
        pool = pool or ModelPool.from_dicts(models, prog.var_names, prog.var_widths)
        out = {}
        # all shapes (the shipped default) and none (MG_BV_FUSE=0)
        for fuse in ("5", "0"):
            monkeypatch.setenv("MG_BV_FUSE", fuse)
            out[fuse] = dev.eval_bits(prog, pool)
        for k in range(3):
            assert np.array_equal(out["5"][k], out["0"][k])
        rfs, rsc = eval_batch(prog, pool)
        assert np.array_equal(out["5"][0], rfs) and np.array_equal(out["5"][1], rsc)
        assert 0 < int(out["5"][1].sum()) < prog.n_dags * pool.n_models
