"""BoundedLoopsStrategy on CPU: the loop count pinned on the
reference's own vectors (tests/laser/strategy/test_loop_bound.py), the C oracle's
literal hash against the Python restatement on random traces (including the
lossy overlap of addresses above 255), and oracle lanes that drop exactly where
single-stepping plus the Python count says the reference drops them."""
import random

import numpy as np
import pytest

import loopref
from mythril_amd.lanes import (LaneBatch, LaneShape, MG_HALT_STOP, MG_LOOP_BOUND, MG_RUNNING)
from oracle.evm_ref import OracleEVM, loop_count
from vmtests_util import load_json


def test_loop_count_reference_vectors():
    from mythril_amd.laser import BoundedLoopsStrategy
    vecs = load_json("loop_count.json")
    assert len(vecs) >= 5
    for v in vecs:
        assert loopref.loop_count(v["trace"]) == v["count"]
        assert loop_count(v["trace"]) == v["count"]
        assert BoundedLoopsStrategy.get_loop_count(v["trace"]) == v["count"]


def _random_trace(rng):
    body = [rng.choice([rng.randrange(256), rng.randrange(1 << 16)]) for _ in range(rng.randint(1, 12))]
    pre = [rng.randrange(1 << 16) for _ in range(rng.randint(0, 6))]
    t = pre + body * rng.randint(1, 6) + body[: rng.randint(0, len(body))]
    if rng.random() < 0.3:   # near-copies whose OR-hash may still collide
        k = rng.randrange(len(t))
        t[k] |= rng.choice([1, 0x100, 0x8000])
    if rng.random() < 0.3:
        t += [t[-2], t[-1]] if len(t) >= 2 else []
    return t


def test_c_loop_count_equals_python_restatement():
    rng = random.Random(2718)
    from mythril_amd.laser import BoundedLoopsStrategy
    for _ in range(3000):
        t = _random_trace(rng)
        assert loop_count(t) == loopref.loop_count(t), t
        assert BoundedLoopsStrategy.get_loop_count(t) == loopref.loop_count(t), t


# PUSH1 0 CALLDATALOAD; loop: JUMPDEST PUSH1 1 SWAP1 SUB DUP1 PUSH1 3 JUMPI; STOP
LOOP = bytes.fromhex("600035" "5b" "6001" "90" "03" "80" "6003" "57" "00")


def loop_batch(ns, trace_cap=256):
    b = LaneBatch(LaneShape(n=len(ns), stack_cap=16, mem_cap=32, calldata_cap=32, storage_cap=1,
                            trace_cap=trace_cap))
    for i, n in enumerate(ns):
        b.set_lane(i, calldata=int(n).to_bytes(32, "big"), gas_limit=10 ** 7)
    return b


def expected_drops(code, batch, bound):
    """Single-step the oracle without a bound; at every JUMPDEST apply the Python
    loop count to the addresses executed so far.  Returns per lane the step at
    which the reference drops the state (None if never)."""
    o = OracleEVM()
    cid = o.load_code(code)
    ops, addrs = o.code_table(cid)
    b = batch.copy()
    b.code_id[:] = cid
    traces = [[] for _ in range(b.n)]
    drop = [None] * b.n
    for _ in range(100000):
        live = [i for i in range(b.n) if int(b.status[i]) == MG_RUNNING and drop[i] is None]
        if not live:
            break
        for i in live:
            pc = int(b.pc[i])
            if pc >= ops.size:
                continue
            traces[i].append(int(addrs[pc]))
            if int(ops[pc]) == 0x5B and loopref.loop_count(traces[i]) > bound:
                drop[i] = (int(b.steps[i]), pc, loopref.loop_count(traces[i]))
        o.run(b, first=0, n=b.n, max_steps=1)
    return drop, traces


@pytest.mark.parametrize("bound", [1, 3, 7])
def test_oracle_lanes_drop_where_the_reference_drops(bound):
    ns = list(range(0, 14)) + [40, 2 ** 200]
    b = loop_batch(ns)
    want, traces = expected_drops(LOOP, b, bound)
    o = OracleEVM()
    ref = b.copy()
    ref.code_id[:] = o.load_code(LOOP)
    o.run(ref, loop_bound=bound)
    for i, n in enumerate(ns):
        if want[i] is None:
            assert int(ref.status[i]) == MG_HALT_STOP, (n, int(ref.status[i]))
            assert list(ref.trace[i, : int(ref.trace_len[i])]) == traces[i][:int(ref.trace_len[i])]
        else:
            steps, pc, cnt = want[i]
            assert int(ref.status[i]) == MG_LOOP_BOUND, n
            assert (int(ref.steps[i]), int(ref.pc[i]), int(ref.aux[i])) == (steps, pc, cnt)
            assert list(ref.trace[i, : int(ref.trace_len[i])]) == traces[i]
    assert any(w is None for w in want) and any(w is not None for w in want)
