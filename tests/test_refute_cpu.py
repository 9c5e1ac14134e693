"""mythril_amd/smt/refute.py: the refutations the SAT-only backend may give
(keccak-axiom select rewrite, unit equalities) -- each one checked for the
unsat it claims and against over-reach: a query that has a model (one found
and checked here) is never refuted, and the keccak rewrite needs the keccak
condition among the conjuncts."""
import pytest

from mythril_amd.smt import expr as E
from mythril_amd.smt.expr import And, Array, Concat, K, Not, symbol_factory
from mythril_amd.smt.keccak_manager import keccak_function_manager as km
from mythril_amd.smt.refute import refutes
from mythril_amd.smt.solver import _conjuncts


@pytest.fixture(autouse=True)
def _fresh_keccak():
    km.reset()
    yield
    km.reset()


def bv(v, w=256):
    return symbol_factory.BitVecVal(v, w)


def word(name):
    return symbol_factory.BitVecSym(name, 256)


def mapping_read(storage, key):
    slot = km.create_keccak(Concat(key, bv(1)))
    return storage[slot] & bv(0xFF)


def fresh_storage():
    s = K(256, 256, 0)
    s[bv(0)] = bv(0)                          # the constructor's write to slot 0
    return s


def query(*cs, axioms=True):
    parts = list(cs) + ([km.create_conditions()] if axioms else [])
    return _conjuncts(And(*parts).raw)


def test_fresh_mapping_read_is_refuted():
    st = fresh_storage()
    assert refutes(query(mapping_read(st, word("sender_2")) == bv(1)))


def test_refutation_needs_the_keccak_condition():
    st = fresh_storage()
    assert not refutes(query(mapping_read(st, word("sender_2")) == bv(1), axioms=False))


def test_slot_written_through_another_key_is_not_refuted():
    st = fresh_storage()
    slot = km.create_keccak(Concat(word("addr"), bv(1)))
    st[slot] = bv(1)
    # readable where sender == addr: satisfiable, must not be refuted
    assert not refutes(query(mapping_read(st, word("sender_3")) == bv(1)))


def test_a_concrete_key_inside_the_interval_is_not_skipped():
    from mythril_amd.smt.keccak_manager import PART
    st = fresh_storage()
    x = Concat(word("sender_2"), bv(1))
    km.create_keccak(x)
    km.create_conditions()
    lo = km.interval_hook_for_size[512] * PART
    st[bv((lo + 63) // 64 * 64)] = bv(1)      # a slot the application may equal
    assert not refutes(query(mapping_read(st, word("sender_2")) == bv(1)))


def test_a_registered_concrete_hash_is_not_skipped():
    st = fresh_storage()
    c = Concat(bv(7), bv(1))
    h = km.create_keccak(c)                   # concrete: keccak(7 . 1)
    st[h] = bv(1)
    # keccak(sender . 1) may equal keccak(7 . 1) (sender = 7)
    assert not refutes(query(mapping_read(st, word("sender_2")) == bv(1)))


def test_unit_equalities():
    cv = word("call_value3")
    iszero = E.If(cv == bv(0), bv(1), bv(0))
    assert refutes(query(iszero != bv(0), E.UGT(cv, bv(0)), axioms=False))
    assert refutes(query(cv == bv(1), cv == bv(2), axioms=False))
    assert not refutes(query(iszero != bv(0), E.ULT(cv, bv(5)), axioms=False))
    assert not refutes(query(Not(cv == bv(0)), E.UGT(cv, bv(0)), axioms=False))


def test_ite_wrappers_only_pin_the_branch_they_force():
    """distinct(ite(P, 1, 0), 2) holds whatever P is, so it must not
    pin P's variable: next to cv == 5 the query is sat (cv = 5)."""
    cv = word("call_value3")
    wrapped = E.If(cv == bv(7), bv(1), bv(0))
    assert not refutes(query(wrapped != bv(2), cv == bv(5), axioms=False))
    assert not refutes(query(wrapped == bv(0), cv == bv(5), axioms=False))
    # the forcing forms still pin it
    assert refutes(query(wrapped != bv(0), cv == bv(5), axioms=False))
    assert refutes(query(wrapped == bv(1), cv == bv(5), axioms=False))


def test_array_reads_are_not_folded():
    cd = Array("calldata", 256, 8)
    q = query(cd[bv(0)] == bv(1, 8), word("x") == bv(3), axioms=False)
    assert not refutes(q)


@pytest.mark.parametrize("name", ["killbilly", "exceptions_0.8.0.sol.o"])
def test_no_query_with_a_model_is_refuted(name, monkeypatch, tmp_path):
    """Every query the SAT-only backend answers with a model (seed or guided
    search, checked on kernel 2's oracle) during an analysis -- refutation off, so the search sees them all
    -- is one refutes() leaves alone."""
    import analyze
    import killbilly
    from fnames import use_signature_db
    from mythril_amd.smt import search
    from oracle_device import OracleDevice, OracleK2
    use_signature_db(monkeypatch, tmp_path)
    monkeypatch.setattr(search, "refutes", lambda conj: False)
    orig = search.SatSearchBackend.__call__
    sat = []

    def call(self, constraints, *a):
        m = orig(self, constraints, *a)           # raises when no model is found
        sat.append(refutes(_conjuncts(search.query_raw(constraints))))
        return m
    monkeypatch.setattr(search.SatSearchBackend, "__call__", call)
    if name == "killbilly":
        # two transactions keep it short; the mapping slots are in play
        analyze.analyze(name, None, 2, OracleDevice(), OracleK2(), code=killbilly.creation())
    else:
        analyze.analyze(name, "Exceptions", 2, OracleDevice(), OracleK2())
    assert sat and not any(sat)
