#!/usr/bin/env python3
"""Per-opcode cost of kernel 1 on converged waves: each program repeats one
opcode pattern; every lane runs the same straight-line code, so a wave never
diverges.  Prints cycles per wave-iteration (2.4 GHz) per pattern."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

from mythril_amd.device import GpuDevice  # noqa: E402
from mythril_amd.lanes import LaneBatch, LaneShape  # noqa: E402

REP = 400
PATTERNS = {
    "push1_pop": bytes([0x60, 0x01, 0x50]) * REP,
    "push32_pop": (bytes([0x7F]) + bytes(range(32)) + bytes([0x50])) * REP,
    "dup1_pop": bytes([0x60, 0x07]) + bytes([0x80, 0x50]) * REP,
    "swap1": bytes([0x60, 0x07, 0x60, 0x08]) + bytes([0x90]) * REP,
    "add": bytes([0x60, 0x07]) + bytes([0x80, 0x01]) * REP,
    "and": bytes([0x60, 0x07]) + bytes([0x80, 0x16]) * REP,
    "eq_iszero": bytes([0x60, 0x07]) + bytes([0x80, 0x14, 0x15]) * REP,
    "mul": bytes([0x60, 0x07]) + bytes([0x80, 0x02]) * REP,
    "eq": bytes([0x60, 0x07]) + bytes([0x80, 0x14]) * REP,
    "lt": bytes([0x60, 0x07]) + bytes([0x80, 0x10]) * REP,
    "iszero": bytes([0x60, 0x07]) + bytes([0x15]) * REP,
    "not": bytes([0x60, 0x07]) + bytes([0x19]) * REP,
    "xor": bytes([0x60, 0x07]) + bytes([0x80, 0x18]) * REP,
    "and_iszero": bytes([0x60, 0x07]) + bytes([0x80, 0x16, 0x15]) * REP,
    "eq_not": bytes([0x60, 0x07]) + bytes([0x80, 0x14, 0x19]) * REP,
    "dup_iszero_pop": bytes([0x60, 0x07]) + bytes([0x80, 0x15, 0x50]) * REP,
    "and_and": bytes([0x60, 0x07, 0x80]) + bytes([0x80, 0x16, 0x80]) * REP,
    "div": bytes([0x60, 0x07, 0x7F]) + b"\x13" * 32 + bytes([0x81, 0x81, 0x04, 0x50]) * REP,
    "shr": bytes([0x60, 0x07]) + bytes([0x60, 0x03, 0x1C]) * REP,
    "jumpdest": bytes([0x5B]) * REP,
    "jump": b"".join(bytes([0x5B, 0x61, (i * 5 + 5) >> 8, (i * 5 + 5) & 0xFF, 0x56]) for i in range(REP)) + b"\x5b",
    "mstore_mload": bytes([0x60, 0x07]) + bytes([0x80, 0x60, 0x40, 0x52, 0x60, 0x40, 0x51, 0x50]) * REP,
    "calldataload": bytes([0x60, 0x04, 0x35, 0x50]) * REP,
    "sload": bytes([0x60, 0x01, 0x54, 0x50]) * REP,
    "sha3_64": bytes([0x60, 0x40, 0x60, 0x00, 0x20, 0x50]) * REP,
    "caller_pop": bytes([0x33, 0x50]) * REP,
    "callvalue_pop": bytes([0x34, 0x50]) * REP,
    "cdsize_pop": bytes([0x36, 0x50]) * REP,
    "sstore": bytes([0x60, 0x07, 0x60, 0x01, 0x55]) * REP,
    "jumpi_fall": bytes([0x5B, 0x60, 0x00, 0x60, 0x00, 0x57]) * REP,
    "exp": bytes([0x60, 0x07]) + bytes([0x60, 0x03, 0x0A]) * REP,
}


def main():
    dev = GpuDevice(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    res = {}
    for name, code in PATTERNS.items():
        if only and name not in only:
            continue
        cid = dev.load_code(code)
        b = LaneBatch(LaneShape(n=n, stack_cap=64, mem_cap=256, calldata_cap=68, storage_cap=4))
        for i in range(n):
            b.set_lane(i, code_id=cid, calldata=bytes(68), gas_limit=10 ** 9 - 1)
        dev.alloc(b.shape)
        dev.upload(b)
        dev.step()                        # warm
        ms = []
        for _ in range(3):
            dev.reset()
            st = dev.step()
            ms.append(st.kernel_ms)
        steps = st.lane_steps / n
        kms = min(ms)
        waves = (n + 63) // 64
        waves_per_simd = waves / 1024.0
        cyc = kms * 1e-3 * 2.4e9 / (steps * max(waves_per_simd, 1.0))
        res[name] = {"steps_per_lane": steps, "kernel_ms": kms, "cycles_per_wave_step": round(cyc, 1),
                     "lane_steps_per_s": st.lane_steps / (kms * 1e-3)}
        print(f"{name:14s} steps/lane {steps:7.0f}  {kms:8.3f} ms  {cyc:8.1f} cyc/wave-step  "
              f"{st.lane_steps / (kms * 1e-3) / 1e9:7.2f} G lane-steps/s", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
