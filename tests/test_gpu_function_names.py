"""The dispatcher's function table on the MI355X (mg_code_table, mg_code_fentries)
and the per-lane function-entry record (mg_lane_soa.fent) that LaserEVM maps to
environment.active_function_name (svm.py:549-637).

* the device's instruction table renders the reference's expected easm files
  (tests/golden/easm.json; two with renamed opcodes, one stale, see
  tests/test_function_names_cpu.py) exactly as the host Disassembly does;
* its function-entry flags equal the host table's and the oracle's
  restatement, bit 1 being the next index's;
* C2 lanes (with and without straight-line runs, code staged whole and as a
  prefix) end with the oracle's record, which the CPU tests pin against a
  single-step restatement of the exec loop.  The symbolic lanes' record is
  checked end to end by the co-simulations of tests/test_gpu_symbolic.py, whose
  outcomes now carry each path's function name."""
import json

import numpy as np
import pytest

from fnames import GOLDEN, easm_from_table
from mythril_amd import workloads
from mythril_amd.lanes import LaneBatch, diff_batches
from mythril_amd.laser.disassembly import Disassembly

pytestmark = pytest.mark.gpu

EASM = json.loads((GOLDEN / "easm.json").read_text())
BYTECODES = json.loads((GOLDEN / "bytecodes.json").read_text())


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.device import GpuDevice
    d = GpuDevice(0)
    yield d
    d.close()


def _raw(code):
    return bytes.fromhex(code[2:] if code.startswith("0x") else code)


def test_device_code_table_renders_the_easm_goldens(dev):
    from test_function_names_cpu import STALE, _expected
    for name in sorted(EASM):
        raw = _raw(BYTECODES[name])
        ops, addrs = dev.code_table(dev.load_code(raw))
        text = easm_from_table(ops, addrs, raw)
        assert text == Disassembly(BYTECODES[name]).get_easm(), name
        if name not in STALE:
            assert text == _expected(name), name


def test_device_function_entries_equal_host_and_oracle(dev):
    from oracle.evm_ref import OracleEVM
    o = OracleEVM()
    codes = dict(BYTECODES)
    codes["disassembly.json"] = json.loads((GOLDEN / "disassembly.json").read_text())["code"]
    codes["synthetic"] = "6001146007575b00" + "63aabbccdd14600d575b" + "6001146101005700" + "60021461"
    for name, code in codes.items():
        raw = _raw(code)
        host = np.array(Disassembly(code).function_entries(), dtype=np.uint8)
        d = dev.code_fentries(dev.load_code(raw))
        assert np.array_equal(d & 1, host), name
        assert np.array_equal(d >> 1, np.append(host[1:], 0)), name
        assert np.array_equal(host, o.code_fentries(o.load_code(raw))), name


@pytest.mark.parametrize("variant", ["default", "reg_runs", "no_runs", "prefix"])
def test_c2_lane_function_entry_record_equals_the_oracle(dev, variant, monkeypatch):
    """default: LDS-form straight-line runs (their closing jumps); reg_runs: the
    register form (closing jumps as single dispatches); no_runs: a hook mask
    (on BALANCE, which the code never reaches) turns runs off, every jump goes
    through the fast path or the general handler; prefix: most of the code
    decodes from the code arena (non-staged decode words)."""
    mask = None
    if variant == "reg_runs":
        monkeypatch.setenv("MG_K1_RUNS", "reg")
    elif variant == "no_runs":
        mask = [1 << 0x31, 0, 0, 0]
    elif variant == "prefix":
        monkeypatch.setenv("MG_K1_PD_CAP", "120")
        monkeypatch.setenv("MG_K1_JR_CAP", "300")
    from oracle.evm_ref import OracleEVM
    code = workloads.bytecode("overflow.sol.o")
    cid = dev.load_code(code)
    b = workloads.c2_batch(4096, code_id=cid, stack_cap=64, mem_cap=1024)
    dev.alloc(b.shape)
    dev.upload(b)
    dev.step(mask) if mask else dev.step()
    out = LaneBatch(b.shape)
    dev.download(out)
    o = OracleEVM()
    ocid = o.load_code(code)
    ref = b.copy()
    ref.code_id[:] = ocid
    o.run(ref)
    out.code_id[:] = ocid
    assert not diff_batches(out, ref), diff_batches(out, ref)[:5]
    d = Disassembly(code)
    names = {d.name_at(int(x)) for x in np.unique(out.fent) if int(x) != 0xFFFFFFFF}
    assert names == {"_function_0x18160ddd", "_function_0x70a08231", "_function_0xa3210e87"}
