"""Function-manager records (include/mythgpu.h MG_REC_*) on the oracle: what the
reference registers while a concrete path runs -- keccak_function_manager's
concrete_hashes for every SHA3 of a non-empty slice
(keccak_function_manager.py:95-114) and, for every concrete EXP, the constraint
result == Power(base, exponent) (exponent_function_manager.py:32-47,
instructions.py:624-638) -- logged per lane in execution order, with the
capacity escape the host regrows on."""
import numpy as np

from mythril_amd.keccak import keccak256
from mythril_amd.lanes import (MG_ESC_RECORD, MG_ESCAPE, MG_HALT_STOP, MG_REC_HEADER, LaneBatch,
                               LaneShape)
from oracle.evm_ref import OracleEVM
from vmtests_util import fill_lane, load_vmtests, vm_shape

W0 = bytes(range(0x10, 0x30))
W1 = bytes(range(0xa0, 0xc0))


def push(v: int, n: int = 32) -> bytes:
    return bytes([0x5f + n]) + v.to_bytes(n, "big")


def sha3(off: int, ln: int) -> bytes:
    return push(ln, 2) + push(off, 2) + b"\x20" + b"\x50"          # ... SHA3 POP


def exp(base: int, e: int) -> bytes:
    return push(e) + push(base) + b"\x0a" + b"\x50"                  # ... EXP POP


SLICES = [(0, 64), (3, 5), (1, 1), (7, 33), (0, 0), (30, 4), (60, 100)]
POWERS = [(2, 3), (3, 255), (0, 0), (2 ** 255 + 7, 2 ** 200 + 1), (7, 2 ** 256 - 1)]
PROGRAM = (push(int.from_bytes(W0, "big")) + push(0, 1) + b"\x52" +
           push(int.from_bytes(W1, "big")) + push(32, 1) + b"\x52" +
           b"".join(sha3(o, n) for o, n in SLICES) +
           b"".join(exp(b, e) for b, e in POWERS) + b"\x00")


def expected():
    mem = bytearray(W0 + W1)
    out = []
    for off, ln in SLICES:
        if ln == 0:
            continue                   # get_empty_keccak_hash: nothing registered
        end = off + ln
        if end > len(mem):
            mem.extend(b"\0" * ((end + 31) // 32 * 32 - len(mem)))
        data = bytes(mem[off:end])
        out.append(("keccak", data, int.from_bytes(keccak256(data), "big")))
    for b, e in POWERS:
        out.append(("exp", b, e, pow(b, e, 2 ** 256)))
    return out


def run(rec_cap, code=PROGRAM, n=1):
    o = OracleEVM()
    b = LaneBatch(LaneShape(n=n, stack_cap=64, mem_cap=1024, calldata_cap=32, storage_cap=4,
                            rec_cap=rec_cap))
    for i in range(n):
        b.set_lane(i, code_id=o.load_code(code) if i == 0 else 0, gas_limit=10 ** 7)
    o.run(b)
    return b


def test_records_match_the_reference_registrations():
    b = run(rec_cap=1024)
    assert int(b.status[0]) == MG_HALT_STOP
    assert [r[1:] for r in b.records(0)] == expected()
    steps = [r[0] for r in b.records(0)]
    assert steps == sorted(steps) and steps[0] == 8     # 2 x (PUSH PUSH MSTORE), PUSH PUSH
    words = sum(MG_REC_HEADER + ((len(r[1]) + 3) // 4 if r[0] == "keccak" else 16)
                for r in expected())
    assert int(b.rec_len[0]) == words


def test_no_records_without_capacity():
    a, b = run(rec_cap=0), run(rec_cap=1024)
    for f in ("pc", "sp", "msize", "steps", "gas_min", "gas_max", "status"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert int(a.rec_len[0]) == 0


def test_full_log_escapes_before_the_instruction():
    full = run(rec_cap=1024)
    need = int(full.rec_len[0])
    first = MG_REC_HEADER + 16           # the first record: keccak of 64 bytes
    for cap in (first - 1, first, need - 1):
        b = run(rec_cap=cap)
        assert int(b.status[0]) == MG_ESCAPE
        assert int(b.aux[0]) >> 8 == MG_ESC_RECORD
        assert int(b.aux[0]) & 0xFF in (0x20, 0x0A)
        got = [r[1:] for r in b.records(0)]
        assert got == expected()[: len(got)]
        assert int(b.rec_len[0]) <= cap
        # the escaped instruction did not run: resuming with room finishes the path
        big = LaneBatch(LaneShape(n=1, stack_cap=64, mem_cap=1024, calldata_cap=32, storage_cap=4,
                                  rec_cap=1024))
        for f in ("code_id", "pc", "sp", "msize", "depth", "steps", "flags", "gas_min", "gas_max",
                  "gas_limit", "calldata_len", "storage_count", "rec_len"):
            getattr(big, f)[...] = getattr(b, f)
        big.stack[...] = b.stack
        big.memory[...] = b.memory
        big.rec[0, :cap] = b.rec[0, :cap]
        o = OracleEVM()
        o.load_code(PROGRAM)
        o.run(big)
        assert int(big.status[0]) == MG_HALT_STOP
        assert big.records(0) == full.records(0)
        assert int(big.steps[0]) == int(full.steps[0])
        assert int(big.gas_min[0]) == int(full.gas_min[0])


def test_vmtests_keccak_records_hash_their_inputs():
    vectors = [v for v in load_vmtests() if not v["ignored"]]
    shape = vm_shape(vectors)
    shape.rec_cap = 1 << 16
    b = LaneBatch(shape)
    o = OracleEVM()
    ids = {}
    for i, v in enumerate(vectors):
        if v["code"] not in ids:
            ids[v["code"]] = o.load_code(bytes.fromhex(v["code"]))
        fill_lane(b, i, v, ids[v["code"]])
    o.run(b)
    n_kec = n_exp = 0
    for i in range(b.n):
        for r in b.records(i):
            if r[1] == "keccak":
                n_kec += 1
                assert int.from_bytes(keccak256(r[2]), "big") == r[3]
            else:
                n_exp += 1
                assert pow(r[2], r[3], 2 ** 256) == r[4]
    assert n_kec >= 5 and n_exp >= 10, (n_kec, n_exp)


def test_symbolic_record_kinds_parse_in_log_order():
    """MG_REC_SYMEXP (payload: the Power node) and MG_REC_CDSIZE (result: the
    CODESIZE value pushed) between an EXP record, as k_sym_step writes them
    (include/mythgpu.h): LaneBatch.records returns them in log order."""
    from mythril_amd.lanes import MG_REC_CDSIZE, MG_REC_EXP, MG_REC_SYMEXP, word_to_limbs
    b = LaneBatch(LaneShape(n=2, stack_cap=8, mem_cap=64, calldata_cap=32, storage_cap=4, rec_cap=64))
    words = []

    def head(kind, ln, step, r):
        words.extend([kind, ln, step] + [int(x) for x in word_to_limbs(r)])
    head(MG_REC_CDSIZE, 0, 3, 0x2c9)
    head(MG_REC_SYMEXP, 0, 7, 0)
    words.append(5)
    head(MG_REC_EXP, 0, 9, 256 ** 3)
    words.extend([int(x) for x in word_to_limbs(256)] + [int(x) for x in word_to_limbs(3)])
    b.rec[1, :len(words)] = words
    b.rec_len[1] = len(words)
    assert b.records(1) == [(3, "cdsize", 0x2c9), (7, "symexp", 5), (9, "exp", 256, 3, 256 ** 3)]
    assert b.records(0) == []
