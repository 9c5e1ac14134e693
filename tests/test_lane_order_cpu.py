"""Lane orders of the C2 batch (mythril_amd/lanes.py): bucket_order and
wave_aligned_order are permutations, and a wave of 64 lanes pays for the union
of its lanes' paths -- the per-lane paths come from the CPU oracle stepping the
bench's 65,536 lanes one instruction at a time."""
import numpy as np
import pytest

from mythril_amd import workloads
from mythril_amd.lanes import MG_RUNNING, bucket_order, wave_aligned_order
from oracle.evm_ref import OracleEVM


def _paths(b):
    o = OracleEVM()
    b = b.copy()
    b.code_id[:] = o.load_code(workloads.bytecode("overflow.sol.o"))
    h = np.zeros(b.n, dtype=np.uint64)
    for _ in range(2000):
        live = b.status == MG_RUNNING
        if not live.any():
            break
        h[live] = h[live] * np.uint64(1000003) + b.pc[live].astype(np.uint64) + np.uint64(1)
        o.run(b, max_steps=1)
    return h, b.steps.copy()


def _serial(order, h, steps, wave=64):
    out = []
    for w in range(0, len(order), wave):
        paths = dict(zip(h[order[w:w + wave]].tolist(), steps[order[w:w + wave]].tolist()))
        out.append(sum(paths.values()))
    return np.array(out)


@pytest.fixture(scope="module")
def c2():
    b = workloads.c2_batch(65536, stack_cap=64, mem_cap=4096)
    return (b,) + _paths(b)


def test_orders_are_permutations(c2):
    b = c2[0]
    for o in (bucket_order(b), wave_aligned_order(b, workloads.C2_SELECTORS)):
        assert np.array_equal(np.sort(o), np.arange(b.n))


def test_large_buckets_share_waves_only_with_fall_through_lanes(c2):
    b = c2[0]
    o = wave_aligned_order(b, workloads.C2_SELECTORS)
    sel = (b.calldata[o, 0].astype(np.int64) << 24 | b.calldata[o, 1].astype(np.int64) << 16
           | b.calldata[o, 2].astype(np.int64) << 8 | b.calldata[o, 3])
    key = sel * 256 + b.calldata_len[o]
    filler = (b.calldata_len[o] < 4) | ~np.isin(sel, workloads.C2_SELECTORS)
    for s in workloads.C2_SELECTORS:
        idx = np.flatnonzero(key == s * 256 + 68)
        assert len(idx) >= 64 and idx[-1] - idx[0] + 1 == len(idx)
        waves = slice(idx[0] // 64 * 64, (idx[-1] // 64 + 1) * 64)
        assert np.all((key[waves] == s * 256 + 68) | filler[waves])


def test_wave_aligned_order_shortens_the_longest_wave(c2):
    b, h, steps = c2
    base = _serial(bucket_order(b), h, steps)
    wave = _serial(wave_aligned_order(b, workloads.C2_SELECTORS), h, steps)
    longest = int(steps.max())                      # sendeth's 203-step path
    assert base.max() > longest + 40                # 203 + a 52-step bucket in one wave
    assert wave.max() <= longest + 12               # only a calldata-too-short lane beside it
    assert wave.mean() <= base.mean()
