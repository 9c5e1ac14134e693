"""Kernel 1's LDS plan variants on an MI355X, bit-exact against the oracle.

The library stages a code's pre-decoded instructions, push immediates and jump
targets in LDS when they fit, else a prefix of them (the rest decodes from HBM),
and keeps each lane's first memory bytes in an LDS window.  The runtime
switches the library reads per launch force every layout onto small codes:

* MG_K1_PD_CAP / MG_K1_JR_CAP: staged prefix of n - 1 instructions / n jump
  targets (lanes cross the prefix boundary in both directions, runs stop at it);
* MG_K1_PUSH=global: push immediates read from the code arena;
* MG_K1_MEMWIN: LDS memory window bytes per lane (0 = off; 32 puts the
  window's edge inside the free-memory pointer's word; 1024 covers all of C2's
  memory), with the VMTests' unaligned and straddling memory accesses;
* MG_K1_RUNS=reg: every straight-line run in the register form (the fallback
  for a run whose stack window does not fit the LDS-resident form).
"""
import os

import pytest

from mythril_amd import workloads
from mythril_amd.device import GpuDevice
from mythril_amd.lanes import LaneBatch, diff_batches
from test_gpu_bench_fidelity import _oracle
from test_gpu_lanes import run_both
from vmtests_util import fill_lane, load_vmtests, vm_shape

pytestmark = pytest.mark.gpu

SWITCHES = ("MG_K1_PD_CAP", "MG_K1_JR_CAP", "MG_K1_PUSH", "MG_K1_MEMWIN", "MG_K1_RUNS")


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


@pytest.fixture
def env():
    saved = {k: os.environ.get(k) for k in SWITCHES}
    yield os.environ
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("switches", [
    {"MG_K1_PD_CAP": "100"},
    {"MG_K1_PD_CAP": "200", "MG_K1_JR_CAP": "300"},
    {"MG_K1_JR_CAP": "0"},
    {"MG_K1_PUSH": "global"},
    {"MG_K1_MEMWIN": "0"},
    {"MG_K1_MEMWIN": "32"},
    {"MG_K1_MEMWIN": "1024", "MG_K1_PD_CAP": "150"},
    {"MG_K1_RUNS": "reg"},
])
def test_c2_under_lds_plan_variants(dev, env, switches):
    env.update(switches)
    code = workloads.bytecode("overflow.sol.o")
    b = workloads.c2_batch(16384, code_id=0, seed=7, stack_cap=64, mem_cap=1024, rec_cap=128)
    ref, cov_ref = _oracle([code], b, coverage=True)
    cid = dev.load_code(code)
    gpu_in = b.copy()
    gpu_in.code_id[:] = cid
    dev.alloc(b.shape, coverage=True)
    dev.coverage_clear()
    dev.upload(gpu_in)
    st = dev.step()
    out = LaneBatch(b.shape)
    dev.download(out)
    out.code_id[:] = b.code_id
    diffs = diff_batches(out, ref, limit=20)
    assert not diffs, diffs
    assert st.lane_steps == int(ref.steps.sum())
    assert (dev.coverage(cid) == cov_ref[:dev.n_instr(cid)]).all()


@pytest.mark.parametrize("memwin", ["0", "32", "96", "4096"])
def test_vmtests_under_memory_windows(dev, env, memwin):
    env["MG_K1_MEMWIN"] = memwin
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    b = LaneBatch(vm_shape(vectors))
    codes, index = [], {}
    for i, v in enumerate(vectors):
        if v["code"] not in index:
            index[v["code"]] = len(codes)
            codes.append(bytes.fromhex(v["code"]))
        fill_lane(b, i, v, index[v["code"]])
    out, ref, _ = run_both(dev, codes, b)
    diffs = diff_batches(out, ref)
    assert not diffs, diffs


def test_large_code_staged_prefix_with_runs(dev, env):
    """The 3,523-instruction fixture: 3,523 pre-decoded entries fit (push
    immediates in HBM); with MG_K1_PD_CAP=1500 the upper half decodes from HBM."""
    code = workloads.large_code()
    sels = workloads.dispatch_selectors(code)
    b = workloads.c2_batch(16384, code_id=0, seed=123, stack_cap=1024, mem_cap=4096, rec_cap=128,
                           selectors=sels)
    ref, cov_ref = _oracle([code], b, coverage=True)
    for cap in (None, "1500"):
        if cap:
            env["MG_K1_PD_CAP"] = cap
        cid = dev.load_code(code)
        gpu_in = b.copy()
        gpu_in.code_id[:] = cid
        dev.alloc(b.shape, coverage=True)
        dev.coverage_clear()
        dev.upload(gpu_in)
        st = dev.step()
        out = LaneBatch(b.shape)
        dev.download(out)
        out.code_id[:] = b.code_id
        diffs = diff_batches(out, ref, limit=20)
        assert not diffs, (cap, diffs)
        assert st.lane_steps == int(ref.steps.sum()) > 16384 * 20
        assert (dev.coverage(cid) == cov_ref[:dev.n_instr(cid)]).all()
