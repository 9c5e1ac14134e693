"""Kernel 1 parity on an MI355X: libmythgpu.so (HIP) vs the CPU oracle, bit-exact.

Every test drives the device through the C-ABI (mythril_amd.device -> ctypes ->
libmythgpu.so) and compares the full lane record (pc, sp, msize, depth, status,
aux, steps, gas min/max, stack, memory, storage, return range) with
oracle/evm_ref.c run on identical inputs.
"""
import random

import numpy as np
import pytest

import pysem
from mythril_amd import workloads
from mythril_amd.device import GpuDevice, hook_mask_for
from mythril_amd.lanes import (LaneBatch, LaneShape, MG_HALT_STOP, MG_HOOK, MG_RUNNING,
                               diff_batches)
from oracle.evm_ref import OracleEVM
from vmtests_util import fill_lane, judge, load_vmtests, vm_shape

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


def run_both(dev, codes, batch, hook_mask=None, max_steps=1 << 30, max_depth=0, coverage=False):
    """Load `codes` on both sides, run `batch` on the device and on the oracle."""
    o = OracleEVM()
    dev_ids = [dev.load_code(c) for c in codes]
    orc_ids = [o.load_code(c) for c in codes]
    # code ids are positional on both sides; remap the batch to the device's ids
    dmap = np.array(dev_ids, dtype=np.uint32)
    gpu_in = batch.copy()
    gpu_in.code_id[:] = dmap[batch.code_id]
    ref = batch.copy()
    ref.code_id[:] = np.array(orc_ids, dtype=np.uint32)[batch.code_id]
    dev.alloc(batch.shape, coverage=coverage)
    dev.upload(gpu_in)
    stats = dev.step(hook_mask, max_steps=max_steps, max_depth=max_depth)
    out = LaneBatch(batch.shape)
    dev.download(out)
    out.code_id[:] = batch.code_id
    o.run(ref, hook_mask=hook_mask or (0, 0, 0, 0), max_steps=max_steps, max_depth=max_depth)
    ref.code_id[:] = batch.code_id
    return out, ref, stats


def test_vmtests_device_equals_oracle(dev):
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    shape = vm_shape(vectors)
    b = LaneBatch(shape)
    codes, index = [], {}
    for i, v in enumerate(vectors):
        if v["code"] not in index:
            index[v["code"]] = len(codes)
            codes.append(bytes.fromhex(v["code"]))
        fill_lane(b, i, v, index[v["code"]])
    out, ref, stats = run_both(dev, codes, b)
    diffs = diff_batches(out, ref)
    assert not diffs, diffs
    # and the device meets the reference harness' own assertions
    verdicts = [judge(out, i, v)[0] for i, v in enumerate(vectors)]
    assert verdicts.count("fail") == 0
    assert verdicts.count("pass") == 499
    assert stats.lane_steps == int(out.steps.sum())


@pytest.mark.parametrize("op", sorted(pysem.BINOPS))
def test_arithmetic_device_equals_oracle_and_python(dev, op):
    nargs, fn = pysem.BINOPS[op]
    rng = random.Random(0xA11 + op)
    sp = pysem.special_words()
    rows = [tuple(rng.choice(sp) for _ in range(nargs)) for _ in range(512)]
    rows += [tuple(rng.getrandbits(rng.choice([8, 64, 128, 200, 255, 256])) for _ in range(nargs))
             for _ in range(1536)]
    if op in (0x04, 0x05, 0x06, 0x07, 0x08, 0x09):
        rows += [tuple(division_operand(rng) for _ in range(nargs)) for _ in range(2048)]
    b = LaneBatch(LaneShape(n=len(rows), stack_cap=16, mem_cap=64, calldata_cap=96, storage_cap=4))
    for i, row in enumerate(rows):
        b.set_lane(i, code_id=0, calldata=b"".join(x.to_bytes(32, "big") for x in row),
                   gas_limit=10 ** 6)
    out, ref, _ = run_both(dev, [pysem.op_program(op, nargs)], b)
    assert not diff_batches(out, ref)
    assert (out.status == MG_HALT_STOP).all()
    for i, row in enumerate(rows):
        assert out.storage_dict(i, drop_zero=False)[0] == fn(*row), (hex(op), row)


def division_operand(rng):
    """Operands that reach every branch of the device's Knuth-D division
    (u256.cuh): every divisor length, top-limb ties (qhat = 2^32 - 1), estimates
    that need refinement or an add-back, and wave-mixed quotient lengths."""
    kind = rng.randrange(8)
    bits = rng.randint(1, 256)
    if kind == 0:
        return rng.getrandbits(bits) | (1 << (bits - 1))
    if kind == 1:   # all-ones limbs
        return (1 << bits) - 1
    if kind == 2:   # top limb 0x80000000.., low limbs zero or ones
        k = rng.randint(1, 8)
        return ((1 << 31) << (32 * (k - 1))) | (rng.choice([0, (1 << (32 * (k - 1))) - 1]))
    if kind == 3:   # repeated limb pattern (equal top limbs in u and v)
        limb = rng.getrandbits(32) | (1 << 31)
        return sum(limb << (32 * i) for i in range(rng.randint(1, 8)))
    if kind == 4:   # 2^k +- small
        return max(1, ((1 << rng.randint(1, 255)) + rng.randint(-3, 3)) & pysem.M)
    if kind == 5:   # limbs of 0xffffffff and 0x00000000 mixed
        return sum(rng.choice([0, 0xFFFFFFFF, 1, 0x80000000]) << (32 * i) for i in range(8))
    if kind == 6:
        return rng.getrandbits(256)
    return rng.getrandbits(rng.choice([32, 33, 63, 64, 65, 96, 224, 225]))


@pytest.fixture(scope="module")
def c2():
    return workloads.bytecode("overflow.sol.o")


def test_c2_full_size_device_equals_oracle(dev, c2):
    b = workloads.c2_batch(65536, stack_cap=64, mem_cap=1024)
    out, ref, stats = run_both(dev, [c2], b)
    diffs = diff_batches(out, ref, limit=20)
    assert not diffs, diffs
    assert stats.lane_steps == int(ref.steps.sum()) > 65536 * 50
    assert stats.running == 0


def test_c2_hook_yield_and_resume(dev, c2):
    """Lanes yield before hooked opcodes (SSTORE, SHA3) exactly where the oracle does,
    and a resumed run (hook cleared) lands on the same final state."""
    b = workloads.c2_batch(4096, seed=7, stack_cap=64, mem_cap=1024)
    mask = hook_mask_for([0x55, 0x20])
    out, ref, _ = run_both(dev, [c2], b, hook_mask=mask)
    assert not diff_batches(out, ref)
    assert (out.status == MG_HOOK).sum() > 0
    # resume: clear the hook status and continue without a mask
    for x in (out, ref):
        hooked = x.status == MG_HOOK
        x.status[hooked] = MG_RUNNING
        x.aux[hooked] = 0
    out.code_id[:] = dev.load_code(c2)
    dev.upload(out)
    dev.step()
    out2 = LaneBatch(out.shape)
    dev.download(out2)
    out2.code_id[:] = 0
    o = OracleEVM()
    o.load_code(c2)
    ref.code_id[:] = 0
    o.run(ref)
    assert not diff_batches(out2, ref)


def test_c2_max_steps_slices_equal_one_run(dev, c2):
    b = workloads.c2_batch(2048, seed=11, stack_cap=64, mem_cap=1024)
    out, ref, _ = run_both(dev, [c2], b)
    b.code_id[:] = dev.load_code(c2)
    dev.upload(b)
    for _ in range(1000):
        st = dev.step(max_steps=7)
        if st.running == 0:
            break
    sliced = LaneBatch(b.shape)
    dev.download(sliced)
    sliced.code_id[:] = 0
    assert not diff_batches(sliced, out)


def test_reset_replays_identically(dev, c2):
    b = workloads.c2_batch(8192, seed=3, stack_cap=64, mem_cap=1024)
    dev.load_code(c2)
    cid = len(dev.codes) - 1
    b.code_id[:] = cid
    dev.alloc(b.shape, coverage=True)
    dev.upload(workloads.slim_copy(b))
    dev.step()
    first = LaneBatch(b.shape)
    dev.download(first)
    dev.reset()
    dev.step()
    second = LaneBatch(b.shape)
    dev.download(second)
    assert not diff_batches(first, second)
    cov = dev.coverage(cid)
    assert cov.sum() > 0
    # every lane that halted inside the code halted on a covered instruction
    n = dev.n_instr(cid)
    pcs = first.pc[first.pc < n]
    assert cov[pcs].all()


def test_run_batches_equal_reset_and_step(dev, c2):
    """mg_run_batches (the bench's timed form) = reset + step per batch: every
    batch reports the oracle's step count, the final lanes equal the oracle's,
    and every batch ran to completion."""
    b = workloads.c2_batch(8192, seed=5, stack_cap=64, mem_cap=1024, rec_cap=128)
    o = OracleEVM()
    ref = b.copy()
    ref.code_id[:] = o.load_code(c2)
    o.run(ref)
    b.code_id[:] = dev.load_code(c2)
    dev.alloc(b.shape)
    dev.upload(workloads.slim_copy(b))
    stats = dev.run_batches(4)
    assert len(stats) == 4
    for st in stats:
        assert st.lane_steps == int(ref.steps.sum())
        assert st.running == 0 and st.kernel_ms > 0
    out = LaneBatch(b.shape)
    dev.download(out)
    out.code_id[:] = ref.code_id
    assert not diff_batches(out, ref, limit=20)


def test_c2_bucketed_order_is_a_permutation(dev, c2):
    """The bench uploads lanes in bucket_order; every lane's result is independent
    of its position, so the permuted device run equals the permuted oracle run."""
    from mythril_amd.lanes import bucket_order, permuted
    b = workloads.c2_batch(16384, seed=5, stack_cap=64, mem_cap=1024)
    order = bucket_order(b)
    pb = permuted(b, order)
    out, ref, _ = run_both(dev, [c2], pb)
    assert not diff_batches(out, ref)
    _, ref0, _ = run_both(dev, [c2], b)
    assert not diff_batches(out, permuted(ref0, order))


def _stack_program(rng, depth_target):
    """Random straight-line program that grows the stack past the LDS window and
    shuffles it with DUPn/SWAPn/arithmetic, then stores the top 8 words."""
    code = bytearray()
    depth = 0
    for _ in range(rng.randrange(200, 600)):
        r = rng.random()
        if depth < 2 or (r < 0.35 and depth < depth_target):
            n = rng.randrange(1, 33)
            code += bytes([0x5F + n]) + rng.getrandbits(8 * n).to_bytes(n, "big")
            depth += 1
        elif r < 0.55 and 1 <= depth < depth_target:
            k = rng.randrange(1, min(16, depth) + 1)
            code.append(0x7F + k)          # DUPk
            depth += 1
        elif r < 0.75 and depth >= 2:
            k = rng.randrange(1, min(16, depth - 1) + 1)
            code.append(0x8F + k)          # SWAPk
        elif r < 0.9:
            code.append(rng.choice([0x01, 0x02, 0x03, 0x16, 0x17, 0x18, 0x1B, 0x1C]))
            depth -= 1
        else:
            code.append(0x50)              # POP
            depth -= 1
        if depth > 1000:
            break
    for s in range(min(8, depth)):
        code += bytes([0x60, s, 0x55])     # PUSH1 s; SSTORE (value = top)
    return bytes(code)


def test_deep_stack_window_edges(dev):
    """Stacks that cross the LDS window (slots >= 16 live in HBM) in both directions,
    several codes per block (unstaged decode path) and one code per block."""
    rng = random.Random(0x57AC)
    codes = [_stack_program(rng, t) for t in (8, 15, 16, 17, 18, 24, 40, 100, 400, 1000)
             for _ in range(4)]
    n = 4096
    b = LaneBatch(LaneShape(n=n, stack_cap=1024, mem_cap=64, calldata_cap=32, storage_cap=16))
    for i in range(n):
        # blocks of 256 lanes: first half of the batch mixes codes, second half stages one
        cid = (i % len(codes)) if i < n // 2 else ((i // 256) % len(codes))
        b.set_lane(i, code_id=cid, gas_limit=10 ** 8)
    out, ref, _ = run_both(dev, codes, b)
    assert not diff_batches(out, ref)
    assert (out.sp > 16).any()
    assert (out.steps > 100).mean() > 0.5


# ------------------------------------------------------------ BoundedLoopsStrategy
from test_loop_bound import LOOP, loop_batch  # noqa: E402


def run_both_loop(dev, codes, batch, bound, hook_mask=None):
    dev.set_loop_bound(bound)
    try:
        o = OracleEVM()
        ids = [dev.load_code(c) for c in codes]
        oids = [o.load_code(c) for c in codes]
        g = batch.copy()
        g.code_id[:] = np.array(ids, dtype=np.uint32)[batch.code_id]
        r = batch.copy()
        r.code_id[:] = np.array(oids, dtype=np.uint32)[batch.code_id]
        dev.alloc(batch.shape)
        dev.upload(g)
        dev.step(hook_mask)
        out = LaneBatch(batch.shape)
        dev.download(out)
        out.code_id[:] = batch.code_id
        o.run(r, hook_mask=hook_mask or (0, 0, 0, 0), loop_bound=bound)
        r.code_id[:] = batch.code_id
        return out, r
    finally:
        dev.set_loop_bound(0)


@pytest.mark.parametrize("bound", [1, 3, 10])
def test_loop_bound_device_equals_oracle(dev, bound):
    from mythril_amd.lanes import MG_ESCAPE, MG_LOOP_BOUND
    rng = random.Random(bound)
    ns = [rng.choice([rng.randrange(0, 40), rng.randrange(0, 200), 2 ** 255]) for _ in range(3000)]
    b = loop_batch(ns, trace_cap=96 if bound < 10 else 48)
    out, ref = run_both_loop(dev, [LOOP], b, bound)
    assert not diff_batches(out, ref, limit=20)
    st = out.status
    assert (st == MG_HALT_STOP).sum() > 0
    if bound < 10:
        assert (st == MG_LOOP_BOUND).sum() > 0
    else:
        assert (st == MG_ESCAPE).sum() > 0    # a 48-entry trace fills before 11 iterations


def test_loop_bound_with_hooks_traces_each_pop_once(dev):
    """A lane stopped at a hooked JUMPDEST and resumed with HOOK_ACK is traced
    once: the hook-by-hook run ends where the uninterrupted run ends."""
    from mythril_amd.lanes import MG_LANE_HOOK_ACK
    ns = list(range(0, 9)) * 20
    b = loop_batch(ns, trace_cap=128)
    whole, _ = run_both_loop(dev, [LOOP], b, 3)
    mask = hook_mask_for([0x5B])
    cur, ref = run_both_loop(dev, [LOOP], b, 3, hook_mask=mask)
    assert not diff_batches(cur, ref)
    for _ in range(200):
        if not (cur.status == MG_HOOK).any():
            break
        for x in (cur, ref):
            h = x.status == MG_HOOK
            x.status[h] = MG_RUNNING
            x.flags[h] |= np.uint32(MG_LANE_HOOK_ACK)
        cur, ref2 = run_both_loop(dev, [LOOP], cur, 3, hook_mask=mask)
        o = OracleEVM()
        o.load_code(LOOP)
        ref.code_id[:] = 0
        o.run(ref, hook_mask=mask, loop_bound=3)
        assert not diff_batches(cur, ref)
        for x in (cur, ref):
            x.flags[:] &= ~np.uint32(MG_LANE_HOOK_ACK)
    for f in ("status", "pc", "steps", "trace_len", "aux"):
        assert np.array_equal(getattr(cur, f), getattr(whole, f)), f


def test_loop_bound_vmtests_and_c2(dev, c2):
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    shape = vm_shape(vectors)
    shape.trace_cap = 4096
    b = LaneBatch(shape)
    codes, index = [], {}
    for i, v in enumerate(vectors):
        if v["code"] not in index:
            index[v["code"]] = len(codes)
            codes.append(bytes.fromhex(v["code"]))
        fill_lane(b, i, v, index[v["code"]])
    out, ref = run_both_loop(dev, codes, b, 3)
    assert not diff_batches(out, ref, limit=20)
    cb = workloads.c2_batch(8192, seed=99, stack_cap=64, mem_cap=1024)
    cb2 = LaneBatch(LaneShape(n=cb.n, stack_cap=64, mem_cap=1024, calldata_cap=96, storage_cap=16,
                              trace_cap=512))
    for f in ("code_id", "pc", "status", "calldata_len", "storage_count", "gas_limit",
              "calldata", "env", "storage"):
        getattr(cb2, f)[...] = getattr(cb, f)
    out, ref = run_both_loop(dev, [c2], cb2, 2)
    assert not diff_batches(out, ref, limit=20)


# ---- function-manager records (MG_REC_*): Keccak registrations and EXP constraints
def test_records_device_equals_oracle(dev):
    from test_records import PROGRAM, expected
    caps = [0, 26, 27, 60, 100, 1024]
    b = LaneBatch(LaneShape(n=len(caps) * 64, stack_cap=64, mem_cap=1024, calldata_cap=32,
                            storage_cap=4, rec_cap=1024))
    for i in range(b.n):
        b.set_lane(i, gas_limit=10 ** 7)
    out, ref, _ = run_both(dev, [PROGRAM], b)
    assert not diff_batches(out, ref)
    assert [r[1:] for r in out.records(0)] == expected()
    # every capacity: the same escape point and the same partial log
    for cap in caps:
        s = LaneBatch(LaneShape(n=64, stack_cap=64, mem_cap=1024, calldata_cap=32, storage_cap=4,
                                rec_cap=cap))
        for i in range(64):
            s.set_lane(i, gas_limit=10 ** 7)
        out, ref, _ = run_both(dev, [PROGRAM], s)
        diffs = diff_batches(out, ref)
        assert not diffs, (cap, diffs)


def test_records_vmtests_and_c2(dev, c2):
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    shape = vm_shape(vectors)
    shape.rec_cap = 1 << 12
    b = LaneBatch(shape)
    codes, index = [], {}
    for i, v in enumerate(vectors):
        if v["code"] not in index:
            index[v["code"]] = len(codes)
            codes.append(bytes.fromhex(v["code"]))
        fill_lane(b, i, v, index[v["code"]])
    out, ref, _ = run_both(dev, codes, b)
    diffs = diff_batches(out, ref)
    assert not diffs, diffs
    b = workloads.c2_batch(65536, stack_cap=64, mem_cap=1024, rec_cap=128)
    out, ref, _ = run_both(dev, [c2], b)
    diffs = diff_batches(out, ref, limit=20)
    assert not diffs, diffs
    assert int(out.rec_len.astype(np.int64).sum()) > 65536 * 10


def test_reupload_into_used_lanes_equals_oracle(dev):
    """Uploads move only the rows below each range's largest sp / msize / storage
    count / trace / record length: a batch uploaded into lanes that held deeper
    states must run exactly as on fresh lanes (no stale row is ever read)."""
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    shape = vm_shape(vectors)
    codes, index = [], {}
    for v in vectors:
        if v["code"] not in index:
            index[v["code"]] = len(codes)
            codes.append(bytes.fromhex(v["code"]))
    first = LaneBatch(shape)
    for i, v in enumerate(vectors):
        fill_lane(first, i, v, index[v["code"]])
    # the same vectors in reverse lane order: every lane gets another vector's state
    second = LaneBatch(shape)
    for i, v in enumerate(reversed(vectors)):
        fill_lane(second, i, v, index[v["code"]])
    ids = np.array([dev.load_code(c) for c in codes], dtype=np.uint32)
    dev.alloc(shape)
    a = first.copy()
    a.code_id[:] = ids[first.code_id]
    dev.upload(a)
    dev.step()
    b = second.copy()
    b.code_id[:] = ids[second.code_id]
    dev.upload(b)                                   # same allocation, lanes dirty
    dev.step()
    out = LaneBatch(shape)
    dev.download(out)
    out.code_id[:] = second.code_id
    o = OracleEVM()
    oids = np.array([o.load_code(c) for c in codes], dtype=np.uint32)
    ref = second.copy()
    ref.code_id[:] = oids[second.code_id]
    o.run(ref, hook_mask=(0, 0, 0, 0))
    ref.code_id[:] = second.code_id
    assert diff_batches(out, ref) == []
