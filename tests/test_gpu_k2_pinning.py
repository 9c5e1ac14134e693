"""Kernel 2 on an MI355X, pinned on the reference's own SMT test data
(tests/k2_pins.py): keccak_tests.py's sat/unsat verdicts through
KeccakFunctionManager.create_conditions -> compile_sets -> k_bv_eval, the
instruction tests' shift rows and EIP-145 tables as programs.  The device must
equal the oracle (oracle/bv_ref.c) bit-exactly and both must match the
reference's verdicts."""
import numpy as np
import pytest

from k2_pins import adversarial_pool, keccak_cases, shift_cases, witness
from mythril_amd.device import GpuDevice
from mythril_amd.smt.flatten import compile_sets
from mythril_amd.smt.program import ModelPool
from oracle.bv_ref import eval_batch

pytestmark = pytest.mark.gpu
NO = 0xFFFFFFFF


@pytest.fixture(scope="module")
def dev():
    d = GpuDevice(0)
    yield d
    d.close()


def test_keccak_cases_on_device(dev):
    for case in keccak_cases():
        prog, kept = compile_sets([case.constraints])
        assert kept == [0]
        models = adversarial_pool(case, 4095, seed=len(case.name))
        if case.expected == "sat":
            models.append(witness(case))
        pool = ModelPool.from_dicts(models, prog.var_names, prog.var_widths, prog.tables)
        fs, sc, bits, _ = dev.eval_bits(prog, pool)
        rfs, rsc = eval_batch(prog, pool)
        assert (fs[0], sc[0]) == (rfs[0], rsc[0]), case.name
        assert int(np.unpackbits(bits[0].view(np.uint8)).sum()) == sc[0]
        if case.expected == "sat":
            last = len(models) - 1
            assert (int(bits[0][last >> 6]) >> (last & 63)) & 1, f"{case.name}: witness rejected"
        else:
            assert fs[0] == NO and sc[0] == 0, f"{case.name}: model {fs[0]} satisfies an unsat query"


def test_shift_rows_on_device(dev):
    cases = shift_cases()
    prog, kept = compile_sets([[c[1]] for c in cases])
    assert kept == list(range(len(cases)))
    pool = ModelPool.from_dicts([c[2] for c in cases], prog.var_names, prog.var_widths)
    fs, sc, bits, _ = dev.eval_bits(prog, pool)
    rfs, rsc = eval_batch(prog, pool)
    assert np.array_equal(fs, rfs) and np.array_equal(sc, rsc)
    for d, (name, _, _, truth) in enumerate(cases):
        assert bool((int(bits[d][d >> 6]) >> (d & 63)) & 1) == truth, name
