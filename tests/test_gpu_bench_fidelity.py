"""The benchmark's exact configuration, parity-tested as a whole (MI355X):

* C2 as bench.py runs it — 65,536 lanes, stack_cap 1,024, bucketed lane order,
  rec_cap 128, coverage on, mg_run_batches from a slim resident image — every
  lane's full record (including its function-manager records) bit-exact against
  the oracle, and the coverage bytes equal to the oracle's;
* the reference's 3,523-instruction disassembler fixture
  (disassembler_test.py:8-10), past the kernel's 1,023-instruction LDS
  pre-decode, stepped with random calldata over its 16 selectors.
"""
import json
from pathlib import Path

import numpy as np
import pytest

from mythril_amd import workloads
from mythril_amd.device import GpuDevice
from mythril_amd.lanes import LaneBatch, bucket_order, diff_batches, permuted
from oracle.evm_ref import OracleEVM

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


def _oracle(codes, batch, coverage=False):
    o = OracleEVM()
    ids = [o.load_code(c) for c in codes]
    ref = batch.copy()
    ref.code_id[:] = np.array(ids, dtype=np.uint32)[batch.code_id]
    cov = None
    if coverage:
        cov = np.zeros(max(o.code_table(ids[0])[0].size, 1), dtype=np.uint8)
        o.set_coverage(ids[0], cov)
    o.run(ref)
    o.set_coverage(ids[0], None)
    ref.code_id[:] = batch.code_id
    return ref, cov


def test_bench_configuration_equals_oracle(dev):
    code = workloads.bytecode("overflow.sol.o")
    cid = dev.load_code(code)
    b = workloads.c2_batch(65536, code_id=0, stack_cap=1024, mem_cap=1024, rec_cap=128)
    b = permuted(b, bucket_order(b))
    ref, ref_cov = _oracle([code], b, coverage=True)
    gpu_in = b.copy()
    gpu_in.code_id[:] = cid
    dev.alloc(b.shape, coverage=True)
    dev.coverage_clear()
    dev.upload(workloads.slim_copy(gpu_in))
    stats = dev.run_batches(2)
    assert all(st.running == 0 and st.lane_steps == int(ref.steps.sum()) for st in stats)
    out = LaneBatch(b.shape)
    dev.download(out)
    out.code_id[:] = b.code_id
    diffs = diff_batches(out, ref, limit=20)
    assert not diffs, diffs
    assert np.array_equal(dev.coverage(cid), ref_cov[:dev.n_instr(cid)])
    assert int(out.rec_len.sum()) > 0


def test_disassembler_fixture_code_on_device(dev):
    fx = json.loads((GOLDEN / "disassembly.json").read_text())
    code = bytes.fromhex(fx["code"][2:])
    cid = dev.load_code(code)
    assert dev.n_instr(cid) == fx["instructions"] == 3523
    sels = workloads.dispatch_selectors(code)
    assert len(sels) == 16
    b = workloads.c2_batch(16384, code_id=0, seed=99, stack_cap=1024, mem_cap=4096,
                           selectors=sels)
    b.flags[:] = 0
    ref, _ = _oracle([code], b)
    gpu_in = b.copy()
    gpu_in.code_id[:] = cid
    dev.alloc(b.shape)
    dev.upload(gpu_in)
    st = dev.step()
    out = LaneBatch(b.shape)
    dev.download(out)
    out.code_id[:] = b.code_id
    diffs = diff_batches(out, ref, limit=20)
    assert not diffs, diffs
    assert st.lane_steps == int(ref.steps.sum()) > 16384 * 20
