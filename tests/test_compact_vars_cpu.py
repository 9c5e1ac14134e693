"""program.compact_vars: a persistent compiler's batch renumbered to the
variables and tables its programs read must evaluate exactly as the full batch
(kernel 2's C oracle on pools built from the same model dicts), and the pool
built for it holds only those variables."""
import numpy as np

from mythril_amd.smt.expr import UGT, Function, If, symbol_factory
from mythril_amd.smt.flatten import Compiler, batch_from
from mythril_amd.smt.program import FuncInterp, ModelPool, compact_vars, read_sets
from oracle_device import OracleK2


def _models(n=300, seed=4):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        m = {f"v{i}": int(rng.integers(0, 9)) for i in range(12)}
        m["f"] = FuncInterp(int(rng.integers(0, 3)), {(int(rng.integers(0, 9)),): 5})
        m["g"] = FuncInterp(1, {(3,): int(rng.integers(0, 9))})
        out.append(m)
    return out


def test_compacted_batches_evaluate_as_the_full_batch():
    v = [symbol_factory.BitVecSym(f"v{i}", 256) for i in range(12)]
    k = symbol_factory.BitVecVal
    f, g = Function("f", [256], 256), Function("g", [256], 256)
    c = Compiler()
    # the compiler sees every variable and both functions first (a long analysis)
    warm = [UGT(v[i] + v[(i + 1) % 12], k(7, 256)).raw for i in range(12)] + \
           [(f(v[0]) == k(5, 256)).raw, (g(v[1]) == k(2, 256)).raw]
    for w in warm:
        c.compile(w)
    # a later launch reads three variables and one function
    later = [UGT(v[3], v[7]).raw, (g(v[9]) == k(4, 256)).raw,
             (If(UGT(v[3], k(4, 256)), v[9], v[7]) == k(2, 256)).raw]
    full = batch_from(c, [c.compile(x) for x in later])
    small = compact_vars(full)
    assert len(full.var_names) == 12 and sorted(small.var_names) == ["v3", "v7", "v9"]
    assert len(full.tables) == 2 and len(small.tables) == 1
    models = _models()
    k2 = OracleK2()
    got = [k2.eval_bits(b, ModelPool.from_dicts(models, b.var_names, b.var_widths, b.tables))[2]
           for b in (full, small)]
    assert np.array_equal(got[0], got[1])
    assert got[0].any()
    # the full batch over a pool that serialises only what it reads (the model
    # cache's head block beside the cached seed columns)
    reads = read_sets(full)
    assert reads == ({full.var_names.index(n) for n in ("v3", "v7", "v9")}, {full.tables.index(small.tables[0])})
    part = ModelPool.from_dicts(models, full.var_names, full.var_widths, full.tables, reads=reads)
    assert not part.values[full.var_names.index("v0")].any()
    assert np.array_equal(k2.eval_bits(full, part)[2], got[0])


def test_a_batch_reading_everything_is_returned_as_is():
    v = [symbol_factory.BitVecSym(f"v{i}", 256) for i in range(3)]
    c = Compiler()
    b = batch_from(c, [c.compile(UGT(v[0] + v[1], v[2]).raw)])
    assert compact_vars(b) is b
