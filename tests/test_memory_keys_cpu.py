"""Memory at symbolic offsets keys its bytes by simplify(index) (memory.py:
117-203): the host's memory_key folds an add chain's constants and puts the
other operands in a canonical order, so an index and its commuted form are
one key, as z3's simplify makes them (state.py memory_key)."""
from mythril_amd.laser.state import Memory, memory_key
from mythril_amd.smt.expr import symbol_factory

BVV = symbol_factory.BitVecVal


def sym(name):
    return symbol_factory.BitVecSym(name, 256)


def test_commuted_operands_are_one_key():
    a, b, c = sym("a"), sym("b"), sym("c")
    assert memory_key((a + b).raw) is memory_key((b + a).raw)
    assert memory_key((a + b + c + BVV(3, 256)).raw) is memory_key((BVV(1, 256) + c + b + BVV(2, 256) + a).raw)
    assert memory_key((a + b).raw) is not memory_key((a + c).raw)


def test_a_word_written_at_a_plus_b_reads_back_at_b_plus_a():
    a, b = sym("a"), sym("b")
    m = Memory()
    v = sym("v")
    m.write_word_at(a + b, v)
    got = m.get_word_at(b + a)
    assert got.raw is v.raw or repr(got) == repr(v), got
    byte = m[b + a + BVV(31, 256)]
    assert repr(byte) == repr(m[a + b + BVV(31, 256)])


def test_constants_fold_into_one_trailing_term():
    a = sym("a")
    k = memory_key((BVV(4, 256) + a + BVV(28, 256)).raw)
    assert k is memory_key((a + BVV(32, 256)).raw)
    assert memory_key((a + BVV(0, 256)).raw) is a.raw
