#!/usr/bin/env python3
"""Where kernel 1's C2 launch time goes, per wave: runs the bench's C2 batch
(65,536 lanes, bucketed order, coverage on) through the diagnostic library
built with -DMG_K1_CLOCKS (ab/clk.so, MYTHGPU_LIB) and prints the shader-clock
cycles per opcode bin for the slowest waves and for the mean wave.
Bins: opcode byte = dispatch iterations that executed it (fast path or general
handler), 256 = straight-line runs (bins pack cycles in bits 0-23 and
iterations in bits 24-31), 257 = prologue, 258 = epilogue,
259 = loop overhead of iterations in which this wave advanced nothing."""
import ctypes
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("MYTHGPU_LIB", "ab/clk.so")
import numpy as np  # noqa: E402

from mythril_amd import workloads  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.lanes import bucket_order, permuted  # noqa: E402

BINS = 262
NAMES = {0x01: "ADD", 0x02: "MUL", 0x03: "SUB", 0x04: "DIV", 0x10: "LT", 0x11: "GT", 0x14: "EQ",
         0x15: "ISZERO", 0x16: "AND", 0x19: "NOT", 0x1C: "SHR", 0x20: "SHA3", 0x33: "CALLER",
         0x34: "CALLVALUE", 0x35: "CDLOAD", 0x36: "CDSIZE", 0x39: "CODECOPY", 0x50: "POP", 0x51: "MLOAD",
         0x52: "MSTORE", 0x54: "SLOAD", 0x55: "SSTORE", 0x56: "JUMP", 0x57: "JUMPI", 0x5B: "JUMPDEST",
         0xF3: "RETURN", 0xFD: "REVERT", 0x00: "STOP", 256: "runs", 257: "prologue", 258: "epilogue",
         259: "idle-iter", 260: "dispatch-head", 261: "fetch"}


def name(b):
    if b in NAMES:
        return NAMES[b]
    if 0x60 <= b <= 0x7F:
        return f"PUSH{b - 0x5F}"
    if 0x80 <= b <= 0x8F:
        return f"DUP{b - 0x7F}"
    if 0x90 <= b <= 0x9F:
        return f"SWAP{b - 0x8F}"
    return hex(b)


def show(title, row, top=18):
    tot = row.sum()
    order = np.argsort(-row)[:top]
    print(f"{title}: {tot:.0f} cycles ({tot / 2.4e3:.1f} us at 2.4 GHz)")
    print("   " + "  ".join(f"{name(int(b))}:{row[b] / tot * 100:.1f}%" for b in order if row[b] > 0))


def main(n=65536):
    dev = GpuDevice(0)
    lib = dev.lib
    lib.mg_k1_clocks.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]
    cid = dev.load_code(workloads.bytecode("overflow.sol.o"))
    batch = workloads.c2_batch(n, code_id=cid, seed=workloads.C2_SEED, stack_cap=1024, mem_cap=1024)
    batch = permuted(batch, bucket_order(batch))
    dev.alloc(batch.shape, coverage=True)
    dev.upload(workloads.slim_copy(batch))
    dev.run_batches(2)
    st = dev.run_batches(1)
    buf = (ctypes.c_uint32 * (4096 * BINS))()
    assert lib.mg_k1_clocks(dev.ctx, buf, 4096 * BINS) == 0
    waves = (n + 63) // 64
    raw = np.frombuffer(buf, dtype=np.uint32).reshape(4096, BINS)[:waves]
    clk = (raw & 0xFFFFFF).astype(np.float64)          # cycles (bits 0-23)
    cnt = (raw >> 24).astype(np.float64)               # iterations (bits 24-31)
    tot = clk.sum(axis=1)
    print(f"launch {st.kernel_ms if hasattr(st, 'kernel_ms') else st}: waves {waves}, cycles/wave "
          f"mean {tot.mean():.0f} p50 {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} max {tot.max():.0f}")
    show("mean wave", clk.mean(axis=0))
    slow = np.argsort(-tot)[:16]
    show("16 slowest waves (mean)", clk[slow].mean(axis=0))
    for w in slow[:4]:
        show(f"wave {w}", clk[w], top=12)
    for title, rows in (("mean wave", slice(None)), ("16 slowest waves", slow)):
        c, k = clk[rows].mean(axis=0), cnt[rows].mean(axis=0)
        order = [b for b in np.argsort(-c)[:14] if k[b] > 0]
        print(f"{title}: iterations per wave {k.sum():.1f}; per bin iterations x cycles/iteration")
        print("   " + "  ".join(f"{name(int(b))}:{k[b]:.1f}x{c[b] / k[b]:.0f}" for b in order))


if __name__ == "__main__":
    main()
