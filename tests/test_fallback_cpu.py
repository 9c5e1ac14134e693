"""The SMT fallback around kernel 2 on CPU:

* SMT-LIB 2 rendering of queries (mythril_amd/smt/smtlib.py): an independent
  S-expression evaluator in this file reads the rendered text back and must
  agree with the DAG's own evaluation on random constraint sets (parity
  unpinned against z3's printer: z3 is absent);
* --solver-log: every backend query lands in the log directory
  (support/model.py:62-73);
* solver_process_backend with a stand-in solver process;
* get_models: speculative parallel backend calls, answers identical to the
  sequential get_model loop (LRU and memo included);
* DelayConstraintStrategy (constraint_strategy.py:19-47) and the fork filter
  of svm.py:319-326 in the batched LaserEVM on the oracle device."""
import random
import sys
from pathlib import Path

import pytest

from mythril_amd.smt import solver, smtlib
from mythril_amd.smt.expr import And, ULT, symbol_factory
from mythril_amd.smt.program import ArrayInterp, FuncInterp
from mythril_amd.smt.semantics import apply_op
from mythril_amd.smt.solver import Constraints, Model, ModelCache, UnsatError
from smt_eval import evaluate
from test_smt_programs import _random_constraints, _random_table_constraints, _random_table_models

BVS, BVV = symbol_factory.BitVecSym, symbol_factory.BitVecVal


# ------------------------------------------------------------ an SMT-LIB reader
def _parse(text):
    toks = text.replace("(", " ( ").replace(")", " ) ").split()
    pos = 0

    def rd():
        nonlocal pos
        t = toks[pos]
        pos += 1
        if t == "(":
            out = []
            while toks[pos] != ")":
                out.append(rd())
            pos += 1
            return out
        return t
    forms = []
    while pos < len(toks):
        forms.append(rd())
    return forms


_OPS = {"bvadd", "bvsub", "bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvand", "bvor",
        "bvxor", "bvshl", "bvlshr", "bvashr", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle",
        "bvsgt", "bvsge", "bvnot", "bvneg"}


class _Eval:
    def __init__(self, decls, model):
        self.sorts = {}
        for d in decls:
            name = d[1].strip("|")
            self.sorts[name] = (d[2], d[3])
        self.model = model

    def width(self, sort):
        return 1 if sort == "Bool" else int(sort[2])

    def ev(self, e):
        """-> (value, width); arrays -> (default, entries)."""
        if isinstance(e, str):
            if e in ("true", "false"):
                return int(e == "true"), 1
            if e.startswith("#b"):
                return int(e[2:], 2), len(e) - 2
            if e.startswith("#x"):
                return int(e[2:], 16), 4 * (len(e) - 2)
            name = e.strip("|")
            args, sort = self.sorts[name]
            if isinstance(sort, list) and sort[0] == "Array":
                it = self.model.get(name)
                return ((it.default, dict(it.entries)) if isinstance(it, ArrayInterp) else (0, {})), 0
            w = self.width(sort)
            v = self.model.get(name, 0)
            return (v if isinstance(v, int) else 0) & ((1 << w) - 1), w
        head = e[0]
        if isinstance(head, list):                      # indexed ops / as const
            if head[0] == "_":
                kind = head[1]
                v, w = self.ev(e[1])
                if kind == "extract":
                    hi, lo = int(head[2]), int(head[3])
                    return (v >> lo) & ((1 << (hi - lo + 1)) - 1), hi - lo + 1
                k = int(head[2])
                return apply_op(kind, w + k, [v], [w], k), w + k
            if head[0] == "as":                          # ((as const (Array ..)) v)
                v, _ = self.ev(e[1])
                return (v, {}), 0
        if head == "_":
            return int(e[1][2:]), int(e[2])
        if head == "ite":
            c, _ = self.ev(e[1])
            return self.ev(e[2] if c else e[3])
        if head in ("and", "or"):
            vals = [self.ev(x)[0] for x in e[1:]]
            return (int(all(vals)) if head == "and" else int(any(vals))), 1
        if head == "not":
            return 1 - self.ev(e[1])[0], 1
        if head == "xor":
            return self.ev(e[1])[0] ^ self.ev(e[2])[0], 1
        if head == "=>":
            return int((not self.ev(e[1])[0]) or self.ev(e[2])[0]), 1
        if head in ("=", "distinct"):
            a, b = self.ev(e[1])[0], self.ev(e[2])[0]
            return int((a == b) == (head == "=")), 1
        if head == "select":
            (d, ent), _ = self.ev(e[1])
            i, _ = self.ev(e[2])
            return ent.get(i, d), int(self.sorts_of_array(e[1]))
        if head == "store":
            (d, ent), _ = self.ev(e[1])
            i, _ = self.ev(e[2])
            v, _ = self.ev(e[3])
            ent = dict(ent)
            ent[i] = v
            return (d, ent), 0
        if head == "concat":
            a, wa = self.ev(e[1])
            b, wb = self.ev(e[2])
            return (a << wb) | b, wa + wb
        if head in _OPS:
            vals = [self.ev(x) for x in e[1:]]
            w = vals[0][1]
            out_w = 1 if head[2:] in ("ult", "ule", "ugt", "uge", "slt", "sle", "sgt", "sge") else w
            return apply_op(head, out_w, [v for v, _ in vals], [x for _, x in vals], None), out_w
        name = head.strip("|")                          # uninterpreted function
        args, sort = self.sorts[name]
        vals = tuple(self.ev(x)[0] for x in e[1:])
        it = self.model.get(name)
        w = self.width(sort)
        v = it.entries.get(vals, it.else_value) if isinstance(it, FuncInterp) else 0
        return v & ((1 << w) - 1), w

    def sorts_of_array(self, arr):
        while isinstance(arr, list):
            if isinstance(arr[0], list) and arr[0][0] == "as":     # ((as const (Array D R)) v)
                return int(arr[0][2][2][2])
            arr = arr[1]
        sort = self.sorts[arr.strip("|")][1]
        return int(sort[2][2])


def _smt_truth(text, model):
    forms = _parse(text)
    decls = [f for f in forms if f[0] == "declare-fun"]
    ev = _Eval(decls, model)
    return int(all(ev.ev(f[1])[0] for f in forms if f[0] == "assert"))


def test_smt2_rendering_reads_back_to_the_same_truth():
    rng = random.Random(31)
    n_true = 0
    for k in range(120):
        cs = _random_table_constraints(rng) if k % 2 else _random_constraints(rng, rng.randrange(1, 5))
        text = smtlib.to_smt2(cs)
        assert text.strip().endswith("(get-model)") and "(check-sat)" in text
        for m in _random_table_models(rng, 3, None):
            m.setdefault("z", rng.getrandbits(256))
            m.setdefault("cd4", rng.getrandbits(8))
            want = evaluate(And(*cs).raw, m)
            assert _smt_truth(text, m) == want, text
            n_true += want
    assert n_true > 10


def test_solver_log_writes_every_backend_query(tmp_path, monkeypatch):
    monkeypatch.setattr(solver, "model_cache", ModelCache(device=object()))
    monkeypatch.setattr(solver.args, "solver_log", str(tmp_path / "log"))
    x = BVS("x", 256)
    seen = []

    def backend(cs, mn, mx, t):
        seen.append(cs)
        return Model({"x": 3})
    solver.set_solver_backend(backend)
    try:
        solver.get_model((ULT(x, BVV(7, 256)),), minimize=(x,))
        files = list((tmp_path / "log").glob("*.smt2"))
        assert len(files) == 1 and "(minimize x)" in files[0].read_text()
        assert "(assert (bvult x (_ bv7 256)))" in files[0].read_text()
    finally:
        solver.set_solver_backend(solver._no_backend)


def test_solver_process_backend_with_a_stand_in_solver(tmp_path):
    stub = tmp_path / "fake_solver.py"
    stub.write_text("import sys\nq = sys.stdin.read()\n"
                    "print('unsat' if 'bv99 256' in q else 'sat')\n"
                    "print('(model (define-fun x () (_ BitVec 256) #x05) (define-fun b () Bool true))')\n")
    be = smtlib.solver_process_backend([sys.executable, str(stub)])
    x = BVS("x", 256)
    m = be([ULT(x, BVV(7, 256))], (), (), 5000)
    assert m["x"] == 5 and m["b"] == 1
    with pytest.raises(UnsatError):
        be([x == BVV(99, 256)], (), (), 5000)


def test_get_models_speculation_equals_the_sequential_loop(monkeypatch):
    """Backend calls run ahead on a pool; the answers, the backend-call order of
    USED answers and the final LRU order equal the sequential get_model loop."""
    class _Dev:                       # kernel 2 stand-in: host evaluation of the pool
        def eval(self, prog, pool):
            raise AssertionError("compiled path not used here")

    def run(parallel):
        solver.get_model.cache_clear()
        mc = ModelCache(device=object())
        # quick-sat on the host (ModelRef.eval) stands in for kernel 2
        def qs(expr):
            key = expr.raw if hasattr(expr, "raw") else expr
            hit, val = mc._memo_get(key)
            if hit:
                return val
            res = False
            for m in reversed(list(mc.model_cache.lru_cache.keys())):
                if m.eval(key, model_completion=True).param == 1:
                    res = mc._select(m)
                    break
            mc._memo_put(key, res)
            return res
        mc.check_quick_sat = qs
        monkeypatch.setattr(solver, "model_cache", mc)
        calls = []

        def backend(cs, mn, mx, t):
            calls.append(len(cs))
            v = {"x": 5 + len(cs)}
            return Model(v)
        solver.set_solver_backend(backend)
        x = BVS("x", 256)
        qs_ = [Constraints([ULT(x, BVV(6 + k, 256))] * (1 + k % 3)) for k in range(12)]
        out = solver.get_models(qs_) if parallel else [solver.get_model(q) for q in qs_]
        lru = [m["x"] for m in mc.model_cache.lru_cache]
        return [o["x"] for o in out], lru
    try:
        assert run(True) == run(False)
    finally:
        solver.set_solver_backend(solver._no_backend)
        solver.get_model.cache_clear()


class _HostModelCache(ModelCache):
    """ModelCache whose quick-sat evaluates the cached models on the host
    (ModelRef.eval) in place of kernel 2: test stand-in, same LRU and memo."""

    def check_quick_sat(self, expr):
        key = expr.raw if hasattr(expr, "raw") else expr
        hit, val = self._memo_get(key)
        if hit:
            return val
        res = False
        for m in reversed(list(self.model_cache.lru_cache.keys())):
            if m.eval(key, model_completion=True).param == 1:
                res = self._select(m)
                break
        self._memo_put(key, res)
        return res

    def check_quick_sat_many(self, queries):
        return [self.check_quick_sat(q) for q in queries]


def test_delay_constraint_strategy_parks_until_the_work_list_empties(monkeypatch):
    from mythril_amd.laser.state import GlobalState, WorldState
    from mythril_amd.laser.strategy import DelayConstraintStrategy
    from mythril_amd.smt.expr import FALSE, Bool as SBool

    class _S:
        def __init__(self, ok):
            self.world_state = WorldState(constraints=[] if ok else [SBool(FALSE)])
            self.mstate = type("M", (), {"depth": 0})()
    monkeypatch.setattr(solver, "model_cache", _HostModelCache(device=object()))
    solver.get_model.cache_clear()
    states = [_S(True), _S(False), _S(True)]
    wl = list(states)
    st = DelayConstraintStrategy(wl, 10 ** 9)
    # the strategy's own cache starts empty: every quick-sat misses -> all parked,
    # then the parked states run one at a time once they get a model
    monkeypatch.setattr(st.model_cache, "check_quick_sat_many", lambda qs: [False] * len(qs))
    assert st.drain() == [states[0]]
    assert len(st.model_cache.model_cache.lru_cache) == 1        # the model joined its cache
    assert st.drain() == [states[2]]                             # states[1] is unsat: dropped
    assert st.drain() == [] and st.pending_worklist == []


def test_fork_filter_at_escapes_prunes_impossible_successors(monkeypatch):
    """svm.py:319-326: when the escape handler (the reference's execute_state)
    returns a fork, only successors with possible constraints are kept."""
    from creation_util import call, deploy  # noqa: F401
    from mythril_amd import workloads
    from mythril_amd.laser import Account, Disassembly, LaserEVM, WorldState, execute_message_call
    from mythril_amd.smt.expr import FALSE, Bool as SBool
    from oracle_device import OracleDevice
    monkeypatch.setattr(solver, "model_cache", _HostModelCache(device=object()))
    solver.get_model.cache_clear()
    seen = []

    def handler(s):
        from copy import copy
        a, b = copy(s), copy(s)
        b.world_state.constraints.append(SBool(FALSE))
        a.mstate.pc = b.mstate.pc = 10 ** 6                     # past the end: ends the path
        seen.append(s)
        return [a, b]
    ws = WorldState()
    acct = Account(workloads.CONTRACT, concrete_storage=True)
    acct.code = Disassembly("6000430000")      # PUSH1 0, NUMBER (escapes: symbolic), ...
    ws.put_account(acct)
    vm = LaserEVM(requires_statespace=False, device=OracleDevice(), escape_handler=handler)
    vm.open_states = [ws]
    execute_message_call(vm, workloads.CONTRACT, workloads.ATTACKER, workloads.ATTACKER, b"",
                         8_000_000, 0, 0)
    assert len(seen) == 1
    assert len(vm.open_states) == 1           # the FALSE branch was pruned before running
