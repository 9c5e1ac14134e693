"""Kernel 1's per-wave Keccak result cache (lane_step.cuh, KC_E entries per
wave): SHA3 results must be bit-exact with oracle/evm_ref.c whether a dispatch
hits in every lane, misses in some, evicts entries, or hashes inputs the cache
does not take (unaligned offset, length other than 64).  Records on and off."""
import random

import pytest

from mythril_amd.device import GpuDevice
from mythril_amd.keccak import keccak_int
from mythril_amd.lanes import MG_HALT_STOP, LaneBatch, LaneShape, diff_batches
from test_gpu_lanes import run_both

pytestmark = pytest.mark.gpu


def _sha3(off, ln, slot):
    # PUSH1 ln PUSH1 off SHA3 PUSH1 slot SSTORE
    return bytes([0x60, ln, 0x60, off, 0x20, 0x60, slot, 0x55])


def program():
    c = bytes([0x60, 0x00, 0x35, 0x60, 0x00, 0x52,     # mem[0:32]  = calldata word 0
               0x60, 0x20, 0x35, 0x60, 0x20, 0x52])    # mem[32:64] = calldata word 1
    c += _sha3(0, 64, 0) + _sha3(0, 64, 1)             # miss, then hit
    for k in range(6):                                 # 6 new keys: evicts the 4-entry cache
        c += bytes([0x60, k, 0x60, 0x20, 0x52]) + _sha3(0, 64, 2 + k)
    c += bytes([0x60, 0x20, 0x35, 0x60, 0x20, 0x52])   # original key again (evicted)
    c += _sha3(0, 64, 8) + _sha3(1, 64, 9) + _sha3(0, 63, 10) + _sha3(4, 64, 11) + _sha3(0, 64, 12)
    return c + b"\x00"


@pytest.mark.parametrize("rec_cap", [0, 512])
def test_keccak_cache_equals_oracle(rec_cap):
    dev = GpuDevice(0)
    try:
        rng = random.Random(0x4B43)
        n = 64 * 16
        b = LaneBatch(LaneShape(n=n, stack_cap=32, mem_cap=1024, calldata_cap=64, storage_cap=16,
                                rec_cap=rec_cap))
        cds = []
        for i in range(n):
            w = i // 64
            if w % 4 == 0:      # whole wave shares one input: every dispatch hits after the first
                cd = (7).to_bytes(32, "big") + w.to_bytes(32, "big")
            elif w % 4 == 1:    # a few distinct inputs per wave: partial hits
                cd = (5).to_bytes(32, "big") + (i % 3).to_bytes(32, "big")
            elif w % 4 == 2:    # one odd lane per wave
                cd = (9).to_bytes(32, "big") + (int(i % 64 == 17)).to_bytes(32, "big")
            else:
                cd = rng.getrandbits(256).to_bytes(32, "big") + rng.getrandbits(256).to_bytes(32, "big")
            cds.append(cd)
            b.set_lane(i, calldata=cd, gas_limit=10 ** 7)
        out, ref, _ = run_both(dev, [program()], b)
        assert not diff_batches(out, ref)
        assert (out.status == MG_HALT_STOP).all()
        for i in (0, 70, 64 * 2 + 17, 64 * 3 + 5):
            st = out.storage_dict(i, drop_zero=False)
            mem = bytearray(cds[i])
            assert st[0] == st[1] == st[8] == st[12] == keccak_int(bytes(mem))
            assert st[9] == keccak_int(bytes(mem[1:64]) + b"\x00")
            assert st[10] == keccak_int(bytes(mem[:63]))
    finally:
        dev.close()
