"""Kernel 1 at 32 and 16 lanes per wave (MG_LANES_PER_WAVE, read by mg_open):
the same bit-exact parity against oracle/evm_ref.c as the default 64.

The lane -> thread mapping, the workgroup's LDS stack-window stride and the
launch grid all change with the width, so the C2 batch, every VMTest and the
deep-stack window edges are re-run through a context opened at each width.
"""
import os
import random

import pytest

from mythril_amd import workloads
from mythril_amd.device import GpuDevice
from mythril_amd.lanes import LaneBatch, LaneShape, diff_batches
from test_gpu_lanes import _stack_program, run_both
from vmtests_util import fill_lane, load_vmtests, vm_shape

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[32, 16])
def narrow_dev(request):
    old = os.environ.get("MG_LANES_PER_WAVE")
    os.environ["MG_LANES_PER_WAVE"] = str(request.param)
    try:
        d = GpuDevice(0)
    finally:
        if old is None:
            del os.environ["MG_LANES_PER_WAVE"]
        else:
            os.environ["MG_LANES_PER_WAVE"] = old
    yield d
    d.close()


def test_c2_and_vmtests_equal_oracle(narrow_dev):
    c2 = workloads.bytecode("overflow.sol.o")
    b = workloads.c2_batch(65536, stack_cap=64, mem_cap=1024)
    out, ref, stats = run_both(narrow_dev, [c2], b)
    assert not diff_batches(out, ref, limit=20)
    assert stats.lane_steps == int(ref.steps.sum())
    assert stats.running == 0

    vectors = [v for v in load_vmtests() if not v["ignored"]]
    vb = LaneBatch(vm_shape(vectors))
    codes, index = [], {}
    for i, v in enumerate(vectors):
        if v["code"] not in index:
            index[v["code"]] = len(codes)
            codes.append(bytes.fromhex(v["code"]))
        fill_lane(vb, i, v, index[v["code"]])
    out, ref, _ = run_both(narrow_dev, codes, vb)
    assert not diff_batches(out, ref)


def test_deep_stack_window_edges(narrow_dev):
    rng = random.Random(0x57AD)
    codes = [_stack_program(rng, t) for t in (8, 15, 16, 17, 24, 100, 1000) for _ in range(3)]
    n = 2048
    b = LaneBatch(LaneShape(n=n, stack_cap=1024, mem_cap=64, calldata_cap=32, storage_cap=16))
    for i in range(n):
        cid = (i % len(codes)) if i < n // 2 else ((i // 64) % len(codes))
        b.set_lane(i, code_id=cid, gas_limit=10 ** 8)
    out, ref, _ = run_both(narrow_dev, codes, b)
    assert not diff_batches(out, ref)
    assert (out.sp > 8).any()
