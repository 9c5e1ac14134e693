"""Algorithmic work of a lane-step batch and its roofline fraction.

The per-unit figures are SURVEY §8(d)'s cost table, applied to the opcode
histogram the device itself counts in a profiling pass (mg_step_profile — the
InstructionProfiler plugin's per-opcode counts as native counters):

* int32 ops of a lane-step: PUSH/DUP/SWAP/POP 8; ADD/SUB 16; AND/OR/XOR/NOT 8;
  compares 16; MUL 192 (w(w+1)/2 mul_lo + w(w-1)/2 mul_hi + 2w^2 adds, w=8);
  DIV/MOD/SDIV/SMOD 2048 (32 w^2); ADDMOD/MULMOD 3 divisions + add/mul; shifts,
  BYTE, SIGNEXTEND 24 (3w); SHA3 8,900 per 136-byte Keccak block; SLOAD/SSTORE
  16 per storage entry compared; everything else 8; plus 4 per step for gas.
* bytes of a lane-step: 32 x (words popped + pushed) + memory bytes touched
  (MLOAD/MSTORE 32, MSTORE8 1, CALLDATALOAD 32, *COPY size, SHA3 length) + 64 per
  SLOAD/SSTORE + 1 opcode byte + push-immediate bytes.

Peaks (MI355X_MICROARCH.md): HBM 8.0 TB/s; INT32 VALU 256 CU x 4 SIMDs x 32
lanes/clk (a wave64 VALU instruction issues over 2 cycles) x 2.4 GHz = 78.6 T
ops/s, the integer counterpart of the guide's 157.3 TF f32 vector peak.  The
dominant kernel's fraction is the larger one.  Next to the nominal peaks every
roofline also carries the sustained ones the box measured with
scripts/probes/peaks.hip (profiles/<round>/peaks.json): 16-byte streaming
reads, and 16 independent add/xor chains per lane at 8 waves per SIMD.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

HBM_PEAK_GBS = 8000.0
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # 78.64
PROFILES = Path(__file__).resolve().parent.parent / "profiles"


def sustained_peaks():
    """(HBM read GB/s, INT32 T ops/s) measured on the box by
    scripts/probes/peaks.hip, newest round first; (None, None) if absent."""
    for f in sorted(PROFILES.glob("r*/peaks.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
            return float(d["hbm_read_gbs"]), float(d["int32_tops"])
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def with_sustained(roof: dict) -> dict:
    """Add peak_sustained / frac_sustained for the roofline's bound."""
    hbm, valu = sustained_peaks()
    peak = hbm if roof.get("priced_as", roof["bound"]) == "hbm" else valu
    if peak:
        roof["peak_sustained"] = peak
        roof["frac_sustained"] = roof["achieved"] / peak
        roof["peak_sustained_source"] = "scripts/probes/peaks.hip (profiles/*/peaks.json)"
    return roof


def _tables():
    ops = np.full(256, 8.0)
    words = np.zeros(256)            # words popped + pushed
    extra_bytes = np.zeros(256)
    for b in (0x01, 0x03):
        ops[b] = 16
    ops[0x02] = 192
    for b in (0x04, 0x05, 0x06, 0x07):
        ops[b] = 2048
    ops[0x08] = 3 * 2048 + 16
    ops[0x09] = 3 * 2048 + 192
    ops[0x0A] = 16 * 192
    for b in (0x0B, 0x1A, 0x1B, 0x1C, 0x1D):
        ops[b] = 24
    for b in range(0x10, 0x16):
        ops[b] = 16
    for b in (0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07, 0x0A, 0x0B, 0x10, 0x11, 0x12, 0x13, 0x14,
              0x16, 0x17, 0x18, 0x1A, 0x1B, 0x1C, 0x1D):
        words[b] = 3
    for b in (0x15, 0x19, 0x35, 0x51, 0x54):
        words[b] = 2
    words[0x08] = words[0x09] = 4
    words[0x20] = 3
    for b in (0x30, 0x32, 0x33, 0x34, 0x36, 0x38, 0x3A, 0x3D, 0x45, 0x58, 0x59):
        words[b] = 1
    for b in (0x37, 0x39, 0x3E):
        words[b] = 3
    words[0x50] = 1
    words[0x52] = words[0x53] = words[0x55] = 2
    words[0x56] = 1
    words[0x57] = 2
    words[0xF3] = words[0xFD] = 2
    for k in range(32):
        words[0x60 + k] = 1
        extra_bytes[0x60 + k] = k + 1
    for k in range(16):
        words[0x80 + k] = 2
        words[0x90 + k] = 4
    for k in range(5):
        words[0xA0 + k] = 2 + k
    extra_bytes[0x35] = 32
    extra_bytes[0x51] = extra_bytes[0x52] = 32
    extra_bytes[0x53] = 1
    extra_bytes[0x54] = extra_bytes[0x55] = 64
    return ops, words, extra_bytes


OPS, WORDS, EXTRA_BYTES = _tables()


def algorithmic_work(op_counts: np.ndarray, extra: np.ndarray):
    """(int32 ops, bytes, lane-steps) of a batch from its opcode histogram.
    extra = [sha3 bytes, copy bytes, storage entries scanned, keccak blocks]."""
    c = op_counts.astype(np.float64)
    steps = float(c.sum())
    ops = float((c * OPS).sum()) + 4.0 * steps
    # SHA3: per-block cost instead of the flat 8; SLOAD/SSTORE: per entry compared
    ops += 8900.0 * float(extra[3]) - 8.0 * float(c[0x20])
    ops += 16.0 * float(extra[2])
    byts = float((c * (32.0 * WORDS + EXTRA_BYTES + 1.0)).sum())
    byts += float(extra[0]) + float(extra[1])
    return ops, byts, steps




def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/rNN/traffic.json, written by scripts/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE rocprofv3 passes of the same bench command).
    Returns (bytes, source) or (None, None) when no summary covers the kernel."""
    for d in sorted(PROFILES.glob("r*"), reverse=True):
        f = d / "traffic.json"
        if f.is_file():
            try:
                rec = json.loads(f.read_text()).get(kernel)
            except (OSError, ValueError):
                rec = None
            if rec:
                return float(rec["traffic_bytes"]), str(f.relative_to(PROFILES.parent))
    return None, None


def division_valu():
    """VALU instructions one wave executes per interpreted 256-bit division of
    kernel 2, minus the interpreter's per-instruction overhead (the add/sub
    class's VALU per instruction less its 16 useful ops), from the newest
    profiles/rNN/k2_div_valu.json (scripts/k2_div_valu.py over a rocprofv3
    SQ_INSTS_VALU pass of scripts/k2_opclass.py).  (value, source) or (None, None)."""
    for d in sorted(PROFILES.glob("r*"), reverse=True):
        f = d / "k2_div_valu.json"
        if f.is_file():
            try:
                rec = json.loads(f.read_text())
                return float(rec["valu_per_division"]), str(f.relative_to(PROFILES.parent))
            except (OSError, ValueError, KeyError):
                pass
    return None, None


def lane_step_roofline(dev, batch, code_id, kernel_ms: float) -> dict:
    """Profile one batch (untimed; the resident image is reset first) and price the
    timed kernel's average launch against the HBM and INT32 VALU peaks."""
    dev.reset()
    op_counts, extra = dev.step_profile()
    dev.reset()
    ops, byts, steps = algorithmic_work(op_counts, extra)
    sec = kernel_ms / 1e3 if kernel_ms > 0 else float("nan")
    gbs = byts / sec / 1e9
    tops = ops / sec / 1e12
    hbm_frac = gbs / HBM_PEAK_GBS
    valu_frac = tops / VALU_PEAK_TOPS
    primary_hbm = hbm_frac >= valu_frac
    traffic, traffic_src = pmc_traffic("k_lane_step")
    sq, sq_src = sq_per_wave("k_lane_step")
    traffic_frac = (traffic / sec / 1e9 / HBM_PEAK_GBS) if traffic else None
    roof = with_sustained({
        # SURVEY §8(d) prices a lane-step's stack words as bytes moved; kernel 1
        # keeps them in registers and LDS, so `frac` (algorithmic bytes over the
        # HBM peak) is an accounting fraction.  The measured bound at C2 is
        # latency: one wave per SIMD, half its cycles parked in s_waitcnt
        # (counter_fracs).
        "bound": "latency",
        "frac_basis": ("§8(d) algorithmic bytes / HBM peak" if primary_hbm
                       else "§8(d) algorithmic int32 ops / INT32 VALU peak"),
        "priced_as": "hbm" if primary_hbm else "valu-int32",
        "achieved": gbs if primary_hbm else tops,
        "peak": HBM_PEAK_GBS if primary_hbm else VALU_PEAK_TOPS,
        "unit": "GB/s" if primary_hbm else "T int32-ops/s",
        "frac": hbm_frac if primary_hbm else valu_frac,
        "traffic": traffic,
        "traffic_unit": "bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
        "traffic_source": traffic_src,
        "traffic_frac": traffic_frac,
        "latency_bound": "65,536 lanes = 1,024 waves = one wave per SIMD: the slowest wave's "
                         "dependent dispatch chain sets the launch time (DESIGN.md §3.1)",
        "kernel": "k_lane_step",
        "kernel_ms": kernel_ms,
        "algorithmic_bytes_per_launch": byts,
        "algorithmic_int32_ops_per_launch": ops,
        "bytes_per_lane_step": byts / max(steps, 1.0),
        "int32_ops_per_lane_step": ops / max(steps, 1.0),
        "alt": {"bound": "valu-int32" if primary_hbm else "hbm",
                "achieved": tops if primary_hbm else gbs,
                "peak": VALU_PEAK_TOPS if primary_hbm else HBM_PEAK_GBS,
                "frac": valu_frac if primary_hbm else hbm_frac},
    })
    # what the counters say the kernel uses: measured HBM bytes over the peak,
    # int32 ops over the VALU peak, and the share of wave cycles parked in
    # s_waitcnt (SQ_WAIT_ANY / SQ_WAVE_CYCLES) -- none near 1: latency
    roof["counter_fracs"] = {"hbm_traffic": traffic_frac, "int32_valu": valu_frac,
                             "sq_wait_any": sq.get("wait_any_frac") if sq else None,
                             "sq_issue_stall": sq.get("wait_inst_frac") if sq else None,
                             "sq_source": sq_src}
    floor = issue_floor()
    if floor:
        roof["issue_floor"] = floor
    return roof


def sq_per_wave(kernel: str):
    """The newest committed SQ per-wave summary of `kernel`
    (profiles/rNN/prof/sq_per_wave.json).  (record, source) or (None, None)."""
    for d in sorted(PROFILES.glob("r*"), reverse=True):
        f = d / "prof" / "sq_per_wave.json"
        if f.is_file():
            try:
                rec = json.loads(f.read_text()).get(kernel)
            except (OSError, ValueError):
                rec = None
            if rec:
                return rec, str(f.relative_to(PROFILES.parent))
    return None, None


def issue_floor():
    """Kernel 1's single-batch issue-bound ceiling (a C2 wave
    whose every s_waitcnt were hidden still takes its issue and issue-stall
    cycles): lane-steps/s, from the SQ summary and the launch it was taken on."""
    sq, src = sq_per_wave("k_lane_step")
    if not sq:
        return None
    busy = 1.0 - float(sq["wait_any_frac"])
    return {"busy_frac": busy, "note": "ceiling = measured lane-steps/s / busy_frac at the same launch "
                                       "(waits hidden, issue unchanged)", "source": src}


def issue_rates():
    """Wave-instructions one CU issues per clock at 8 waves per SIMD, per class,
    from the newest profiles/rNN/issue_rates.json (scripts/probes/issue_rates.hip).
    (dict, source) or (None, None)."""
    for f in sorted(PROFILES.glob("r*/issue_rates.json"), reverse=True):
        try:
            r = json.loads(f.read_text())["rates"]
            # the SALU loop carries 3 loop instructions per 16 measured ones
            return ({"salu": r["salu"]["8"]["wave_instr_per_cu_clk"] * 19.0 / 16.0,
                     "valu": r["valu"]["8"]["wave_instr_per_cu_clk"],
                     "branch_pairs": r["branch"]["8"]["wave_instr_per_cu_clk"]},
                    str(f.relative_to(PROFILES.parent)))
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def k2_issue_floor(kernel_ms: float, cus: int = 256, clock_hz: float = 2.4e9):
    """Kernel 2's issue-bound floor on its C4 launch:
    per class, the SQ pass's wave-instructions per launch over one CU's issue
    rate; the floor is the largest, and the launch's measured time over it says
    how close the interpreter runs to issue-bound."""
    sq, sq_src = sq_per_wave("k_bv_eval")
    rates, r_src = issue_rates()
    if not sq or not rates or kernel_ms <= 0:
        return None
    waves = float(sq["SQ_WAVES"])
    per_cu = lambda k: float(sq[k]) * waves / cus
    ms = {"salu": per_cu("SQ_INSTS_SALU") / rates["salu"] / clock_hz * 1e3,
          "valu": per_cu("SQ_INSTS_VALU") / rates["valu"] / clock_hz * 1e3,
          "branch": 2.0 * per_cu("SQ_INSTS_BRANCH") / rates["branch_pairs"] / clock_hz * 1e3}
    bound = max(ms, key=ms.get)
    return {"floor_ms": ms[bound], "bound": bound, "class_ms": ms, "kernel_ms": kernel_ms,
            "frac": ms[bound] / kernel_ms, "sq_source": sq_src, "rates_source": r_src,
            "note": "per-class issue time of the SQ pass's instructions at the probe's rates "
                    "(2.4 GHz assumed for both; the ratio does not depend on it)"}
