"""Synthetic workloads of BASELINE.json's configs.

C2 — "65,536 concrete lanes stepping token.sol bytecode with random calldata":
token.sol cannot be compiled here (no solc), so the code is the precompiled
overflow.sol.o runtime (token.sol with transfer renamed sendeth; compare
solidity_examples/token.sol:1-22 with tests/testdata/input_contracts/overflow.sol).
Lane inputs follow SURVEY §8(d) C2 exactly, from numpy PCG64(seed=0x4D595448).
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from .keccak import keccak_int
from .lanes import (ENV_CALLER, ENV_CALLVALUE, ENV_GASPRICE, ENV_ORIGIN, ENV_ADDRESS, LaneBatch,
                    LaneShape, MG_RUNNING)

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"

ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF   # transaction/symbolic.py:33
CONTRACT = 0x0901D12EBE1B195E5AA8748E62BD7734AE19B51F   # any fixed callee address
C2_SEED = 0x4D595448
C2_SELECTORS = (0x18160DDD, 0x70A08231, 0xA3210E87)     # totalSupply, balanceOf, sendeth


def bytecode_names():
    """The reference's precompiled test contracts (tests/testdata/inputs/*.sol.o)."""
    return list(json.loads((GOLDEN / "bytecodes.json").read_text()))


def bytecode(name: str) -> bytes:
    codes = json.loads((GOLDEN / "bytecodes.json").read_text())
    return bytes.fromhex(codes[name])


def _words_to_limbs(rows: np.ndarray) -> np.ndarray:
    """(n, 32) big-endian bytes -> (n, 8) little-endian u32 limbs."""
    be = rows.reshape(-1, 8, 4).astype(np.uint32)
    dw = (be[:, :, 0] << 24) | (be[:, :, 1] << 16) | (be[:, :, 2] << 8) | be[:, :, 3]
    return dw[:, ::-1].copy()


def large_code() -> bytes:
    """The reference's 3,523-instruction disassembler fixture
    (tests/disassembler_test.py:8-10, tests/golden/disassembly.json): a solc
    runtime with 16 dispatcher selectors, past what fits in LDS with its push
    immediates -- the bench's large-contract field and its parity test."""
    fx = json.loads((GOLDEN / "disassembly.json").read_text())
    code = fx["code"]
    return bytes.fromhex(code[2:] if code.startswith("0x") else code)


def _int_limbs(x: int) -> np.ndarray:
    return np.array([(x >> (32 * k)) & 0xFFFFFFFF for k in range(8)], dtype=np.uint32)


def dispatch_selectors(code: bytes):
    """The 4-byte function selectors of a solc dispatcher: every PUSH4 argument
    compared by an EQ within the next two instructions."""
    from .laser.disassembly import disassemble
    ins = disassemble(code)
    out = []
    for k, i in enumerate(ins):
        if i["opcode"] == "PUSH4" and any(j["opcode"] == "EQ" for j in ins[k + 1:k + 3]):
            v = int(i["argument"], 16)
            if v not in out and v != 0xFFFFFFFF:
                out.append(v)
    return tuple(out)


def c2_batch(n: int = 65536, code_id: int = 0, seed: int = C2_SEED, stack_cap: int = 1024,
             mem_cap: int = 1024, storage_cap: int = 16, gas_limit: int = 8_000_000,
             rec_cap: int = 0, selectors=C2_SELECTORS) -> LaneBatch:
    """SURVEY §8(d) C2 lanes.  `selectors` = the function selectors drawn with
    probability 7/8 (C2: token.sol's three; other codes: dispatch_selectors)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    shape = LaneShape(n=n, stack_cap=stack_cap, mem_cap=mem_cap, calldata_cap=96,
                      storage_cap=storage_cap, rec_cap=rec_cap)
    b = LaneBatch(shape)
    # --- calldata: selector | arg0 | arg1, length 68 w.p. 15/16 else U{0..67}
    sel_known = rng.random(n) < 7 / 8
    sel_pick = rng.integers(0, len(selectors), n)
    sel_rand = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    sel = np.where(sel_known, np.array(selectors, dtype=np.uint64)[sel_pick], sel_rand)
    cd = np.zeros((n, 96), dtype=np.uint8)
    for k in range(4):
        cd[:, k] = (sel >> np.uint64(8 * (3 - k))) & np.uint64(0xFF)
    arg0 = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    addr_like = rng.random(n) < 3 / 4
    arg0[addr_like, :12] = 0
    arg1 = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    small = rng.random(n) < 1 / 2
    arg1[small, :30] = 0
    cd[:, 4:36] = arg0
    cd[:, 36:68] = arg1
    full = rng.random(n) < 15 / 16
    lens = np.where(full, 68, rng.integers(0, 68, n)).astype(np.uint32)
    cd[np.arange(96)[None, :] >= lens[:, None]] = 0
    b.calldata[:, :96] = cd
    b.calldata_len[:] = lens
    # --- environment (transaction/concolic.py:75-122 with the ATTACKER actor)
    b.env[:, ENV_ADDRESS] = _int_limbs(CONTRACT)
    b.env[:, ENV_CALLER] = _int_limbs(ATTACKER)
    b.env[:, ENV_ORIGIN] = _int_limbs(ATTACKER)
    b.env[:, ENV_CALLVALUE] = 0
    b.env[:, ENV_GASPRICE] = _int_limbs(1)
    # --- storage: balances[caller] (mapping at slot 0) and totalSupply (slot 1)
    bal_slot = keccak_int(ATTACKER.to_bytes(32, "big") + (0).to_bytes(32, "big"))
    bal = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    tot = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    b.storage[:, 0, :8] = _int_limbs(bal_slot)
    b.storage[:, 0, 8:] = _words_to_limbs(bal)
    b.storage[:, 1, :8] = _int_limbs(1)
    b.storage[:, 1, 8:] = _words_to_limbs(tot)
    b.storage_count[:] = 2
    # --- machine state
    b.code_id[:] = code_id
    b.status[:] = MG_RUNNING
    b.gas_limit[:] = gas_limit
    return b


def slim_shape(shape: LaneShape) -> LaneShape:
    """Host image that carries no stack/memory contents (fresh lanes): uploads only
    scalars, calldata, env and storage."""
    return LaneShape(n=shape.n, stack_cap=1, mem_cap=32, calldata_cap=shape.calldata_cap,
                     storage_cap=shape.storage_cap)


def slim_copy(batch: LaneBatch) -> LaneBatch:
    out = LaneBatch(slim_shape(batch.shape))
    for f in ("code_id", "pc", "sp", "msize", "depth", "status", "aux", "steps", "flags",
              "calldata_len", "storage_count", "ret_offset", "ret_len", "gas_min", "gas_max",
              "gas_limit"):
        getattr(out, f)[...] = getattr(batch, f)
    out.calldata[...] = batch.calldata
    out.env[...] = batch.env
    out.storage[...] = batch.storage
    return out
