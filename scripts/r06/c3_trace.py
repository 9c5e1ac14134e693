"""Round 6 diagnostic: the all-modules field, contract by
contract, on the oracle device and on the MI355X, with an event trace --
every fork (transaction, instruction address, depth, a structural digest of
the branch condition) and every SAT-backend call (digest of the query,
outcome) -- and the first event where the two runs differ.

    python scripts/r06/c3_trace.py flag_array.sol.o,metacoin.sol.o [--gpu]
"""
import hashlib
import json
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import analyze  # noqa: E402
import fnames  # noqa: E402
from mythril_amd.laser import symbolic as sym  # noqa: E402
from mythril_amd.laser.disassembly import SignatureDB  # noqa: E402
from mythril_amd.smt import search as search_mod  # noqa: E402
from mythril_amd.smt.solver import query_raw  # noqa: E402
from oracle_device import OracleDevice, OracleK2  # noqa: E402

_memo = {}


def digest(n) -> str:
    """Bottom-up structural digest (op, width, param, child digests)."""
    stack = [(n, False)]
    while stack:
        x, done = stack.pop()
        if id(x) in _memo:
            continue
        if done:
            h = hashlib.blake2b(repr((x.op, x.width, x.param, [_memo[id(a)][1] for a in x.args])).encode(),
                                digest_size=8).hexdigest()
            _memo[id(x)] = (x, h)
        else:
            stack.append((x, True))
            stack.extend((a, False) for a in x.args if id(a) not in _memo)
    return _memo[id(n)][1]


EVENTS = []
_orig_succ = sym.jumpi_successors
_orig_call = search_mod.SatSearchBackend.__call__


LIGHT = "--light" in sys.argv


def traced_succ(state):
    st = state.mstate.stack
    cond = st[-2]
    raw = getattr(cond, "raw", None)
    if LIGHT:
        EVENTS.append(("fork", state.current_transaction.id if state.current_transaction else None,
                       state.get_current_instruction()["address"], state.mstate.depth))
    else:
        EVENTS.append(("fork", state.current_transaction.id if state.current_transaction else None,
                       state.get_current_instruction()["address"], state.mstate.depth,
                       digest(raw) if raw is not None else str(cond), repr(raw)[:300]))
    return _orig_succ(state)


import refmodules  # noqa: E402
_orig_exec = refmodules._Base.execute
_orig_gts = refmodules.get_transaction_sequence


def traced_exec(self, target):
    tx = target.current_transaction
    EVENTS.append(("hook", type(self).__name__, target.get_current_instruction()["address"],
                   tx.id if tx else None))
    return _orig_exec(self, target)


def traced_gts(state, constraints):
    tx = state.current_transaction
    EVENTS.append(("gts", state.get_current_instruction()["address"], tx.id if tx else None, len(constraints)))
    return _orig_gts(state, constraints)


traced_exec.__name__ = "execute"      # taint.TaintPlan classifies hooks by module.execute
refmodules._Base.execute = traced_exec
_orig_cpi = refmodules.check_potential_issues
_orig_gpia = refmodules.get_potential_issues_annotation
_lists = {}


def _lid(lst):
    return _lists.setdefault(id(lst), (lst, len(_lists)))[1]


def traced_gpia(state):
    a = _orig_gpia(state)
    EVENTS.append(("pia", state.get_current_instruction()["address"], _lid(a.potential_issues),
                   len(a.potential_issues)))
    return a


def traced_cpi(state):
    a = refmodules.get_potential_issues_annotation.__wrapped__(state) if False else None
    for ann in state.annotations:
        if isinstance(ann, refmodules.PotentialIssuesAnnotation):
            a = ann
    EVENTS.append(("cpi", state.get_current_instruction()["address"],
                   _lid(a.potential_issues) if a else None,
                   [(p.detector.__class__.__name__, p.address) for p in a.potential_issues] if a else []))
    return _orig_cpi(state)


refmodules.get_potential_issues_annotation = traced_gpia
refmodules.check_potential_issues = traced_cpi
refmodules.get_transaction_sequence = traced_gts


def traced_call(self, constraints, minimize, maximize, timeout):
    if LIGHT:
        try:
            m = _orig_call(self, constraints, minimize, maximize, timeout)
            EVENTS.append(("search", len(constraints), "sat"))
            return m
        except Exception as e:
            EVENTS.append(("search", len(constraints), type(e).__name__))
            raise
    key = query_raw(constraints)
    d = hashlib.blake2b("".join(sorted(digest(c) for c in key)).encode(), digest_size=8).hexdigest() \
        if isinstance(key, (list, tuple)) else digest(key)
    try:
        m = _orig_call(self, constraints, minimize, maximize, timeout)
        EVENTS.append(("search", d, "sat"))
        return m
    except Exception as e:
        EVENTS.append(("search", d, type(e).__name__))
        raise


sym.jumpi_successors = traced_succ
search_mod.SatSearchBackend.__call__ = traced_call


TX = 2


def main():
    global TX
    names = sys.argv[1].split(",")
    for a in sys.argv:
        if a.startswith("--tx="):
            TX = int(a[5:])
    d = tempfile.mkdtemp()
    fnames.signature_db(Path(d))
    os.environ["MYTHRIL_DIR"] = d
    SignatureDB._reset()
    import threading

    def beat():                      # a liveness line for the box's silence watchdog
        import time as _t
        while True:
            _t.sleep(30)
            print("...", flush=True, file=sys.stderr)
    threading.Thread(target=beat, daemon=True).start()
    devs = [] if "--only-gpu" in sys.argv else [("cpu", OracleDevice(), OracleK2())]
    if "--gpu" in sys.argv or "--only-gpu" in sys.argv:
        from mythril_amd.device import GpuDevice
        g = GpuDevice(0)
        devs.append(("gpu", g, g))
    out = {}
    for name in names:
        runs = {}
        for tag, dev, k2 in devs:
            EVENTS.clear()
            _memo.clear()
            _lists.clear()
            if name == "BECToken":
                import bectoken
                issues, info = analyze.analyze(name, None, TX, dev, k2, code=bectoken.creation(), search=False)
            else:
                issues, info = analyze.analyze(name, None, TX, dev, k2)
            runs[tag] = {"events": list(EVENTS), "issues": analyze.issue_table(issues),
                         "info": {k: info[k] for k in ("forks", "confirmations", "search", "fork_filter")}}
            print(tag, name, json.dumps(runs[tag]["info"]), flush=True)
        if len(runs) == 2:
            a, b = runs["cpu"]["events"], runs["gpu"]["events"]
            key = lambda e: e[:5] if e[0] == "fork" else e  # noqa: E731
            first = next((i for i in range(min(len(a), len(b))) if key(a[i]) != key(b[i])), None)
            print(name, "events", len(a), len(b), "first difference at", first, flush=True)
            if first is not None:
                for i in range(max(0, first - 3), min(first + 6, max(len(a), len(b)))):
                    print("  ", i, a[i] if i < len(a) else None, "|", b[i] if i < len(b) else None)
        out[name] = runs
    os.makedirs(ROOT / "gpurun_out" / "r06", exist_ok=True)
    with open(ROOT / "gpurun_out" / "r06" / ("c3_trace_%s.json" % names[0].replace(".sol.o", "")), "w") as f:
        json.dump(out, f, default=str)


if __name__ == "__main__":
    main()
