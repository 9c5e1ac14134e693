// lane_step.cuh — kernel 1: batched concrete LASER stepping, one EVM path per lane.
//
// Replaces, for device-eligible paths, the reference hot loop
//   LaserEVM.exec (svm.py:293-337) -> execute_state (svm.py:369-491)
//   -> Instruction.evaluate (instructions.py:235-267) -> StateTransition
//      (instructions.py:98-202) -> opcode mutators (instructions.py:269-1959)
// with the reference's quirks.  Every lane steps until it
// halts, escapes to the host, reaches a hooked opcode or has executed max_steps
// instructions in this launch.  A lane that stops keeps the state it had at the
// start of the stopping instruction (the pre-step state of final_states).
//
// Each opcode handler runs in three phases: (1) pops, checks, memory-extension
// gas and escape decisions, no writes; (2) accumulate_gas + its OOG check
// (instructions.py:162-176) — the only exception the reference raises after a
// mutator has written; (3) writes.
#pragma once
#include "device_state.h"
#include "keccak.cuh"
#include "u256.cuh"

// ---- constants shared with the host side (mythgpu.hip) ----------------------
struct OpInfo {
    uint32_t gmin, gmax;   // support/opcodes.py:16-144 GAS
    uint32_t req;          // STACK[0]: items required by the svm precheck
    uint32_t valid;        // 0 -> disassembles to INVALID
};

#define ST_RUNNING 0u
#define ST_STOP 1u
#define ST_RETURN 2u
#define ST_REVERT 3u
#define ST_END 4u
#define ST_DROPPED 5u
#define ST_VMEXC 6u
#define ST_HOOK 7u
#define ST_ESCAPE 8u
#define ST_DEPTH 9u
#define ST_LOOP 10u

#define EXC_UNDERFLOW 1u
#define EXC_OVERFLOW 2u
#define EXC_BADJUMP 3u
#define EXC_INVALID 4u
#define EXC_OOG 5u
#define EXC_WRITEPROT 6u

#define ESC_OPCODE 1u
#define ESC_MEMORY 2u
#define ESC_STORAGE 3u
#define ESC_STACK 4u
#define ESC_TRACE 5u
#define ESC_RECORD 6u

#define LANE_STATIC 1u
#define LANE_CREATION 2u
#define LANE_HOOK_ACK 4u
#define LANE_STEP1 8u
#define LANE_RETDATA 16384u

#define MSTATE_GAS_LIMIT 1000000000ull
#ifndef MG_K1_PF
#define MG_K1_PF 0
#endif
#define RUN_MAX 64u   // longest straight-line run executed as one block
static_assert(RUN_MAX <= 64u, "a run is read as one pre-decoded word per wave lane");
#define STACK_LIMIT 1024u
#define BIG_END (1ull << 32)
#define HUGE_GAS (1ull << 62)

// ---- lane-interleaved accessors ---------------------------------------------
// Explicit address spaces: DevLanes is a by-value struct argument, so without
// them every access through its pointers would be a flat (generic) access.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_u4;
typedef __attribute__((address_space(3))) v4u l_u4;
typedef __attribute__((address_space(3))) uint32_t l_u32;
template <class T> DEV __attribute__((address_space(1))) T *gp(T *p) {
    return (__attribute__((address_space(1))) T *)p;
}
DEV g_u4 *gv(const void *p) { return (g_u4 *)const_cast<void *>(p); }

DEV U256 ld_word(const g_u4 *base, size_t idx) {
    const v4u x = base[2 * idx], y = base[2 * idx + 1];
    U256 r;
    r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
    r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
    return r;
}
DEV U256 ld_word(const l_u4 *base, size_t idx) {
    const v4u x = base[2 * idx], y = base[2 * idx + 1];
    U256 r;
    r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
    r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
    return r;
}
DEV void st_word(g_u4 *base, size_t idx, const U256 &v) {
    base[2 * idx] = v4u{v.w[0], v.w[1], v.w[2], v.w[3]};
    base[2 * idx + 1] = v4u{v.w[4], v.w[5], v.w[6], v.w[7]};
}
// LDS stack window: slots [0, win) of a lane live in LDS as [slot][half][lane of
// the block] 16-byte pieces (conflict-free ds_read_b128), deeper slots in HBM.
// LDS memory window: memory dwords [0, mw) of a lane live in LDS as [dword][lane
// of the block] (conflict-free at a common offset); HBM holds the rest, and the
// window's bytes once the launch flushes them.  Solidity keeps its scratch words,
// free-memory pointer and first allocation (0x00-0x9f) there.
// `ws` = lanes per block (the row stride), `tid` = the lane's index in its block.
#define LANE_BLOCK 256u
struct LaneView {
    const DevLanes &L;
    uint32_t lane;
    l_u4 *win_base;      // LDS window of this block
    uint32_t win, tid, ws;
    l_u32 *mw_base;      // LDS memory window of this block
    uint32_t mw;         // memory dwords per lane in it
    DEV size_t row(uint32_t r) const { return (size_t)r * L.N + lane; }
    DEV U256 gstack(uint32_t slot) const { return ld_word(gv(L.stack), row(slot)); }
    DEV void set_gstack(uint32_t slot, const U256 &v) const { st_word(gv(L.stack), row(slot), v); }
    DEV U256 wstack(uint32_t slot) const {
        const v4u x = win_base[(slot * 2u) * ws + tid];
        const v4u y = win_base[(slot * 2u + 1u) * ws + tid];
        U256 r;
        r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
        r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
        return r;
    }
    DEV void set_wstack(uint32_t slot, const U256 &v) const {
        win_base[(slot * 2u) * ws + tid] = v4u{v.w[0], v.w[1], v.w[2], v.w[3]};
        win_base[(slot * 2u + 1u) * ws + tid] = v4u{v.w[4], v.w[5], v.w[6], v.w[7]};
    }
    DEV U256 stack(uint32_t slot) const {
        U256 r;
        if (slot < win) r = wstack(slot);
        else r = gstack(slot);
        return r;
    }
    DEV void set_stack(uint32_t slot, const U256 &v) const {
        if (slot < win) set_wstack(slot, v);
        else set_gstack(slot, v);
    }
    DEV U256 env(int w) const { return ld_word(gv(L.env), row((uint32_t)w)); }
    DEV uint32_t lmdw(uint32_t dw) const { return mw_base[dw * ws + tid]; }
    DEV void set_lmdw(uint32_t dw, uint32_t v) const { mw_base[dw * ws + tid] = v; }
    DEV uint32_t gmdw(uint32_t dw) const { return gp(L.mem)[row(dw)]; }
    DEV void set_gmdw(uint32_t dw, uint32_t v) const { gp(L.mem)[row(dw)] = v; }
    DEV uint32_t mdw(uint32_t dw) const { return dw < mw ? lmdw(dw) : gmdw(dw); }
    DEV uint32_t mdw_safe(uint32_t dw) const { return dw < L.mem_cap / 4u ? mdw(dw) : 0u; }
    DEV void set_mdw(uint32_t dw, uint32_t v) const {
        if (dw < mw) set_lmdw(dw, v);
        else set_gmdw(dw, v);
    }
    DEV uint32_t mbyte(uint32_t off) const { return (mdw(off >> 2) >> (24u - 8u * (off & 3u))) & 0xffu; }
    DEV void set_mbyte(uint32_t off, uint32_t b) const {
        const uint32_t sh = 24u - 8u * (off & 3u);
        const uint32_t d = mdw(off >> 2);
        set_mdw(off >> 2, (d & ~(0xffu << sh)) | ((b & 0xffu) << sh));
    }
    // 32 bytes at off (off + 32 <= mem_cap)
    DEV U256 mword(uint32_t off) const {
        U256 r;
        const uint32_t d0 = off >> 2, s = 8u * (off & 3u);
        if (s == 0u && d0 + 8u <= mw) {
#pragma unroll
            for (int k = 0; k < 8; ++k) r.w[7 - k] = lmdw(d0 + k);
        } else if (s == 0u) {
#pragma unroll
            for (int k = 0; k < 8; ++k) r.w[7 - k] = mdw(d0 + k);
        } else {
            uint32_t d[9];
#pragma unroll
            for (int j = 0; j < 9; ++j) d[j] = mdw_safe(d0 + j);
#pragma unroll
            for (int k = 0; k < 8; ++k) r.w[7 - k] = (d[k] << s) | (d[k + 1] >> (32u - s));
        }
        return r;
    }
    DEV void set_mword(uint32_t off, const U256 &v) const {
        const uint32_t d0 = off >> 2, s = 8u * (off & 3u);
        if (s == 0u && d0 + 8u <= mw) {
#pragma unroll
            for (int k = 0; k < 8; ++k) set_lmdw(d0 + k, v.w[7 - k]);
        } else if (s == 0u) {
#pragma unroll
            for (int k = 0; k < 8; ++k) set_mdw(d0 + k, v.w[7 - k]);
        } else {
            const uint32_t keep = 0xffffffffu >> s;   // low bits of the first dword are ours
            const uint32_t first = mdw(d0), last = mdw(d0 + 8);
            set_mdw(d0, (first & ~keep) | (v.w[7] >> s));
#pragma unroll
            for (int j = 1; j < 8; ++j) set_mdw(d0 + j, (v.w[8 - j] << (32u - s)) | (v.w[7 - j] >> s));
            set_mdw(d0 + 8, (v.w[0] << (32u - s)) | (last & keep));
        }
    }
    DEV void mzero(uint32_t from, uint32_t to) const {   // [from, to), multiples of 32
        for (uint32_t dw = from >> 2; dw < (to >> 2); ++dw) set_mdw(dw, 0u);
    }
    DEV uint32_t cdw(uint32_t dw) const { return gp(L.calldata)[row(dw)]; }
    DEV uint32_t cbyte(uint32_t idx) const { return (cdw(idx >> 2) >> (24u - 8u * (idx & 3u))) & 0xffu; }
};

// ---- memory extension (machine_state.py:132-191) -----------------------------
#define MX_OK 0
#define MX_OOG 1
#define MX_ESCAPE 2
// later_min < 0: no OOG check follows in this instruction; otherwise the
// instruction ends with an OOG check after adding later_min gas.
DEV int mem_extend(const U256 &start, const U256 &size, uint32_t &msize, uint64_t &gmin,
                   uint64_t &gmax, uint32_t mem_cap, int64_t later_min, uint64_t txlim) {
    const U256 end = u_add(start, size);
    // python ints do not wrap; anything past 2^32 bytes costs > 1e9 gas
    const bool wrapped = u_lt(end, start);
    if (wrapped || !(end.w[2] == 0u && end.w[3] == 0u && end.w[4] == 0u && end.w[5] == 0u &&
                     end.w[6] == 0u && end.w[7] == 0u))
        return MX_OOG;
    const uint64_t e = (uint64_t)end.w[0] | ((uint64_t)end.w[1] << 32);
    if (e > BIG_END) return MX_OOG;
    if ((uint64_t)msize > e) return MX_OK;
    const uint64_t nw = (e + 31u) >> 5, ow = msize >> 5;
    if (nw == ow) return MX_OK;
    const uint64_t fee = (3u * nw + (nw * nw) / 512u) - (3u * ow + (ow * ow) / 512u);
    const uint64_t nmin = gmin + fee;
    if (nmin > MSTATE_GAS_LIMIT) return MX_OOG;
    if (nw * 32u > mem_cap) {
        if (later_min >= 0 && (nmin + (uint64_t)later_min > MSTATE_GAS_LIMIT ||
                               nmin + (uint64_t)later_min >= txlim))
            return MX_OOG;
        return MX_ESCAPE;
    }
    gmin = nmin;
    gmax += fee;
    msize = (uint32_t)(nw * 32u);
    return MX_OK;
}

DEV bool gas_oog(uint64_t gmin, uint64_t txlim) { return gmin > MSTATE_GAS_LIMIT || gmin >= txlim; }

// Keccak-256 of memory [off, off+len) (off + len <= msize <= mem_cap).  With
// rec != nullptr the input is also copied to the record payload at rec (one
// big-endian word per N-strided row, bytes past len zero).
DEV U256 keccak_mem(const LaneView &V, uint32_t off, uint32_t len, uint32_t *__restrict__ rec = nullptr,
                    size_t N = 0) {
    uint64_t st[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) st[i] = 0ull;
    uint32_t pos = 0;
    const uint32_t s = 8u * (off & 3u);
    // little-endian u64 made of the 8 memory bytes at off + p
    auto le64 = [&](uint32_t p) -> uint64_t {
        const uint32_t dw = (off + p) >> 2;
        const uint32_t a = V.mdw_safe(dw), b = V.mdw_safe(dw + 1u);
        uint32_t be0, be1;
        if (s == 0u) { be0 = a; be1 = b; }
        else {
            const uint32_t c = V.mdw_safe(dw + 2u);
            be0 = (a << s) | (b >> (32u - s));
            be1 = (b << s) | (c >> (32u - s));
        }
        if (rec) {
            const uint32_t w = p >> 2;                       // payload word of be0
            const int32_t v0 = (int32_t)len - (int32_t)p;   // valid bytes from p on
            if (v0 > 0) rec[(size_t)w * N] = v0 >= 4 ? be0 : be0 & ~(0xffffffffu >> (8 * v0));
            if (v0 > 4) rec[(size_t)(w + 1u) * N] = v0 >= 8 ? be1 : be1 & ~(0xffffffffu >> (8 * (v0 - 4)));
        }
        return (uint64_t)__builtin_bswap32(be0) | ((uint64_t)__builtin_bswap32(be1) << 32);
    };
    for (;;) {
        const uint32_t rem = len - pos;
        const bool last = rem < 136u;
#pragma unroll
        for (int j = 0; j < 17; ++j) {
            uint64_t v = 0ull;
            const int32_t nvalid = (int32_t)rem - 8 * j;
            if (nvalid > 0) {
                v = le64(pos + 8u * (uint32_t)j);
                if (nvalid < 8) v &= (1ull << (8 * nvalid)) - 1ull;
            }
            if (last) {
                if (nvalid >= 0 && nvalid < 8) v ^= 0x01ull << (8 * nvalid);
                if (j == 16) v ^= 0x80ull << 56;
            }
            st[j] ^= v;
        }
        keccak_f1600(st);
        if (last) break;
        pos += 136u;
    }
    U256 r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r.w[7 - 2 * q] = __builtin_bswap32((uint32_t)st[q]);
        r.w[6 - 2 * q] = __builtin_bswap32((uint32_t)(st[q] >> 32));
    }
    return r;
}

// ---- function-manager records (include/mythgpu.h MG_REC_*) ----------------------
// Word k of lane `lane`'s record log lives at rec[k * N + lane].  The writers
// fill words from `at` on and return the new length; the caller publishes it
// (rec_len) only when the instruction completes.
DEV uint32_t rec_head(const DevLanes &L, uint32_t lane, uint32_t at, uint32_t kind, uint32_t len, uint32_t step,
                      const U256 &r) {
    uint32_t *__restrict__ q = L.rec + lane;
    const size_t N = L.N;
    q[(size_t)at * N] = kind;
    q[(size_t)(at + 1u) * N] = len;
    q[(size_t)(at + 2u) * N] = step;
#pragma unroll
    for (int k = 0; k < 8; ++k) q[(size_t)(at + 3u + k) * N] = r.w[k];
    return at + MG_REC_HEADER;
}
DEV uint32_t rec_exp(const DevLanes &L, uint32_t lane, uint32_t at, uint32_t step, const U256 &r,
                     const U256 &base, const U256 &exponent) {
    at = rec_head(L, lane, at, MG_REC_EXP, 0u, step, r);
    uint32_t *__restrict__ q = L.rec + lane;
    const size_t N = L.N;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        q[(size_t)(at + k) * N] = base.w[k];
        q[(size_t)(at + 8u + k) * N] = exponent.w[k];
    }
    return at + 16u;
}

// ---- decode table -----------------------------------------------------------------
// One uint2 per opcode byte, built on the host (mythgpu.hip build_decode):
//   x = gas_min | gas_max << 16                  (support/opcodes.py:16-144 GAS)
//   y = req | npop << 4 | push << 8 | kind << 9  (req: svm precheck STACK[0];
//       npop: words the mutator really pops; push: leaves one word; kind: handler)
enum OpKind : uint32_t {
    K_ALU = 0, K_PUSH, K_DUP, K_SWAP, K_LOG, K_POP, K_ENV, K_STOP, K_SHA3, K_CDLOAD, K_CDCOPY,
    K_CODECOPY, K_RDCOPY, K_MLOAD, K_MSTORE, K_MSTORE8, K_SLOAD, K_SSTORE, K_JUMP, K_JUMPI,
    K_JUMPDEST, K_BEGINSUB, K_RETURN, K_REVERT, K_INVALID, K_ESCAPE,
    K_END   // sentinel after the last instruction (past-the-end pc, svm.py:384-389)
};
__constant__ uint2 kDec[256];

// Generic ALU opcodes: res = f(a, b, c) with a the first word popped.
__device__ __forceinline__ U256 alu_slow(uint32_t op, U256 a, U256 b, U256 c) {
    switch (op) {
    case 0x04: return u_iszero(b) ? u_zero() : z_udiv(a, b);            // DIV  (:505-520)
    case 0x05: return u_iszero(b) ? u_zero() : z_sdiv(a, b);            // SDIV (:522-537)
    case 0x06: return u_iszero(b) ? u_zero() : z_urem(a, b);            // MOD  (:539-551)
    case 0x07: return u_iszero(b) ? u_zero() : z_srem(a, b);            // SMOD (:580-592)
    case 0x08: return z_urem(u_add(z_urem(a, c), z_urem(b, c)), c);     // ADDMOD quirk (:594-607)
    case 0x09: return z_urem(u_mul(z_urem(a, c), z_urem(b, c)), c);     // MULMOD quirk (:609-622)
    case 0x0a: return u_exp(a, b);                                      // EXP concrete
    default: return u_zero();
    }
}
DEV U256 alu(uint32_t op, const U256 &a, const U256 &b, const U256 &c) {
    switch (op) {
    case 0x01: return u_add(a, b);
    case 0x02: return u_mul(a, b);
    case 0x03: return u_sub(a, b);
    case 0x0b: {  // SIGNEXTEND with the signed test s0 <= 31 (:640-668)
        const U256 tb = u_add(u_shl_n(a, 3u), u_small(7));
        const U256 set = u_shl(u_small(1), tb);
        const bool sign = !u_iszero(u_and(b, set));
        if (u_slt(u_small(31), a)) return b;
        return sign ? u_or(b, u_neg(set)) : u_and(b, u_sub(set, u_small(1)));
    }
    case 0x10: return u_small(u_lt(a, b));
    case 0x11: return u_small(u_lt(b, a));
    case 0x12: return u_small(u_slt(a, b));
    case 0x13: return u_small(u_slt(b, a));
    case 0x14: return u_small(u_eq(a, b));
    case 0x15: return u_small(u_iszero(a));
    case 0x16: return u_and(a, b);
    case 0x17: return u_or(a, b);
    case 0x18: return u_xor(a, b);
    case 0x19: return u_not(a);
    case 0x1a: {  // BYTE (:426-456)
        U256 r = u_zero();
        if (u_fits32(a) && a.w[0] <= 31u) r.w[0] = u_shr_n(b, (31u - a.w[0]) * 8u, 0u).w[0] & 0xffu;
        return r;
    }
    case 0x1b: return u_shl(b, a);    // value << shift
    case 0x1c: return u_lshr(b, a);
    case 0x1d: return u_ashr(b, a);
    default: return alu_slow(op, a, b, c);
    }
}

// ---- general handlers (one instruction, every opcode kind) ---------------------
// Registers of one lane that an instruction may change.
struct LaneRegs {
    U256 T0, T1;                 // S[sp-1], S[sp-2]
    uint64_t gmin, gmax;
    uint32_t pc, sp, msize, depth;
    uint32_t n_sha3, n_exp;
    uint32_t stop, sx;           // out: ST_RUNNING or the stop status and its aux word
    uint32_t step;               // instructions this launch executed before this one
    uint32_t fent;               // last JUMP / JUMPI landing on a function entry (L.fent)
};
// What the handlers read besides the registers (per lane / per block).
// Per-wave Keccak result cache in LDS (SHA3 of 64 aligned bytes: a mapping
// slot keccak(key . slot), the common case).  Entry e = 16 input dwords + 8 hash
// limbs; word KC_E * 24 holds the valid mask, the next one the replacement index.
#define KC_E 4u
#define KC_WAVE (KC_E * 24u + 2u)
struct StepEnv {
    const DevLanes *L;
    DevCode C;
    const uint8_t *a8;
    const uint32_t *a32;
    l_u4 *s_win;
    l_u32 *s_mw;           // LDS memory window (mw dwords per lane)
    const uint4 *s_pd;     // pre-decoded code: x, y = decode words, z, w = run table
    const uint4 *s_push;
    uint32_t *s_prof;
    uint32_t *s_kc;      // this wave's Keccak cache (KC_WAVE words)
    uint64_t txlim, glim;
    uint32_t lane, tid, ws, win, flags, sflag, psflag, prof;
    uint32_t mw;
    uint32_t sn;         // s_pd holds instructions [0, sn) (the END sentinel included when staged whole)
    uint32_t tosmem;     // the caller keeps the stack's top two words in memory too (k_sym_step):
                         // no spill of T1 below a push
};

// Executes the instruction decoded as (uk, ux) for one lane, exactly as the
// reference would (three phases: checks, accumulate_gas, writes).  The fast
// loop of k_lane_step handles the common opcodes itself and calls this for
// everything else and for any lane whose fast-path preconditions fail, so
// every exception, escape and corner case has a single implementation.
// Inlined (as is alu_slow): a call would need the lane registers and this
// environment in addressable memory, i.e. a scratch frame, and a dispatch with
// scratch pays ~35 us of setup per launch on gfx950 besides the spill traffic.
__device__ __forceinline__ void slow_step(LaneRegs &R, const StepEnv &E, uint32_t uk, uint32_t ux) {
    const DevLanes &L = *E.L;
    const DevCode &C = E.C;
    const uint32_t lane = E.lane;
    const LaneView V{L, lane, E.s_win, E.win, E.tid, E.ws, E.s_mw, E.mw};
    const uint8_t *__restrict__ a8 = E.a8;
    const uint32_t *__restrict__ a32 = E.a32;
    const uint8_t *__restrict__ gops = a8 + C.op_off;
    const uint64_t txlim = E.txlim, glim = E.glim;
    const uint32_t op = uk & 0xffu, kind = (uk >> 17) & 31u;
    const uint32_t req = (uk >> 8) & 15u, npop = (uk >> 12) & 15u;
    const bool push = ((uk >> 16) & 1u) != 0u;
    const uint32_t gtab_min = ux & 0xffffu, gtab_max = ux >> 16;
    const uint32_t sp = R.sp, pc = R.pc, msize0 = R.msize;
    uint32_t nmsize = R.msize, ndepth = R.depth, npc = pc + 1u, nfent = R.fent;
    uint64_t ngmin = R.gmin, ngmax = R.gmax;
    uint32_t stop = ST_RUNNING, sx = 0;
    bool by_table = true;
    const U256 a = R.T0, b = R.T1;
    U256 c = u_zero(), res = u_zero();
    const uint32_t nsp = sp - npop;
    uint32_t *s_prof = E.s_prof;
    const bool prof = E.prof != 0u;
    uint32_t rec_at = 0u, rec_new = 0u;     // function-manager record log (rec_cap > 0)

#define STOPX(s_, x_) { stop = (s_); sx = (x_); break; }
#define EXCX(k_) STOPX(ST_VMEXC, (k_))
#define ESCX(r_) STOPX(ST_ESCAPE, op | ((r_) << 8))
#define GASCOMMIT() if (by_table) { ngmin += gtab_min; ngmax += gtab_max; by_table = false; \
                                    if (ngmin >= glim) EXCX(EXC_OOG) }
#define MEMX(st_, sz_, later_) { const int mx_ = mem_extend((st_), (sz_), nmsize, ngmin, ngmax, \
                                                        L.mem_cap, (later_), txlim); \
                                 if (mx_ == MX_OOG) EXCX(EXC_OOG) if (mx_ == MX_ESCAPE) ESCX(ESC_MEMORY) }
#define ZEROFILL() if (nmsize > msize0) V.mzero(msize0, nmsize);
#define JUMP_OK(idx_) ((idx_) != MG_JRES_NONE && \
                       ((E.sflag && (idx_) < E.sn) ? (E.s_pd[(idx_)].y & 0xffu) : (uint32_t)gops[(idx_)]) == 0x5bu)
    // _new_node_state (svm.py:575-637): a JUMP / JUMPI successor at a function entry
#define FENT_AT(idx_) ((E.sflag && (idx_) < E.sn) ? (E.s_pd[(idx_)].y >> 22) & 1u : a8[C.fent_off + (idx_)] & 1u)

    do {
        // svm.py:391-402 precheck; instructions.py:188-193 write protection;
        // then what the mutator really pops (ADDMOD, SSTORE pop more than `req`)
        if (sp < req) EXCX(EXC_UNDERFLOW)
        if ((op == 0x55u || (op >= 0xa0u && op <= 0xa4u)) && (E.flags & LANE_STATIC)) EXCX(EXC_WRITEPROT)
        if (sp < npop) EXCX(EXC_UNDERFLOW)
        if (npop >= 3u) c = V.stack(sp - 3u);
        bool tos_done = false;
        switch (kind) {
        case K_ALU:
            if (op == 0x0a && L.rec_cap) {
                rec_at = L.rec_len[lane];
                if (rec_at + MG_REC_HEADER + 16u > L.rec_cap) ESCX(ESC_RECORD)
            }
            res = alu(op, a, b, c);
            if (op == 0x0a) {
                ++R.n_exp;
                if (L.rec_cap) rec_new = rec_exp(L, lane, rec_at, L.steps[lane] + R.step, res, a, b);
            }
            break;
        case K_PUSH:                                        // (:278-320)
            res = E.psflag ? ld_word((const l_u4 *)E.s_push, pc)
                           : ld_word(gv(a32 + C.push_off), pc);
            break;
        case K_DUP: {                                       // (:322-331)
            const uint32_t k = op - 0x7fu;
            if (sp < k) EXCX(EXC_UNDERFLOW)
            res = k == 1u ? a : k == 2u ? b : V.stack(sp - k);
            break;
        }
        case K_SWAP: {                                      // (:333-343)
            const uint32_t k = op - 0x8fu;
            if (sp < k + 1u) EXCX(EXC_UNDERFLOW)
            if (k == 1u) {
                GASCOMMIT()
                R.T0 = b; R.T1 = a;
            } else {
                const U256 x = V.stack(sp - 1u - k);
                GASCOMMIT()
                V.set_stack(sp - 1u - k, a);
                R.T0 = x;
            }
            tos_done = true;
            break;
        }
        case K_RDCOPY:                                      // last_return_data None: pops only
            if (E.flags & LANE_RETDATA) ESCX(ESC_OPCODE)
            break;
        case K_LOG: case K_POP: case K_JUMPDEST:
            break;                                          // pops only / no-op
        case K_ENV:
            switch (op) {
            case 0x30: res = V.env(0); break;               // ADDRESS
            case 0x32: res = V.env(2); break;               // ORIGIN
            case 0x33: res = V.env(1); break;               // CALLER
            case 0x34: res = V.env(3); break;               // CALLVALUE
            case 0x3a: res = V.env(4); break;               // GASPRICE
            case 0x36: res = u_small(L.calldata_len[lane]); break;
            case 0x38: res = u_small(C.n_bytes); break;     // CODESIZE
            case 0x45: res = u_small(MSTATE_GAS_LIMIT); break;
            case 0x58: res = u_small(a32[C.addr_off + pc]); break;
            case 0x59: res = u_small(msize0); break;
            default:                                        // RETURNDATASIZE
                if (E.flags & LANE_RETDATA) ESCX(ESC_OPCODE)
                res = u_zero();
                break;
            }
            break;
        case K_STOP: STOPX(ST_STOP, 0u)
        case K_SHA3: {  // own gas first, then mem_extend (instructions.py:1013-1051)
            by_table = false;
            const bool big = (b.w[2] | b.w[3] | b.w[4] | b.w[5] | b.w[6] | b.w[7]) != 0u;
            const uint64_t blen = (uint64_t)b.w[0] | ((uint64_t)b.w[1] << 32);
            const uint64_t g = (big || blen > BIG_END) ? HUGE_GAS : 30ull + 6ull * ((blen + 31ull) >> 5);
            ngmin += g; ngmax += g;
            if (ngmin >= glim) EXCX(EXC_OOG)
            MEMX(a, b, -1)
            if (b.w[0] != 0u && L.rec_cap) {
                rec_at = L.rec_len[lane];
                if ((uint64_t)rec_at + MG_REC_HEADER + ((b.w[0] + 3u) >> 2) > L.rec_cap) ESCX(ESC_RECORD)
            }
            ZEROFILL()
            if (b.w[0] == 0u) {  // get_empty_keccak_hash (keccak_function_manager.py:87-93)
                res.w[7] = 0xc5d24601u; res.w[6] = 0x86f7233cu; res.w[5] = 0x927e7db2u; res.w[4] = 0xdcc703c0u;
                res.w[3] = 0xe500b653u; res.w[2] = 0xca82273bu; res.w[1] = 0x7bfad804u; res.w[0] = 0x5d85a470u;
            } else {
                // Keccak cache: when every lane running this SHA3 finds its 64-byte
                // aligned input among its wave's cached entries (e.g. balances[caller]
                // hashed again), the hashes come from LDS and Keccak-f is skipped; else
                // all lanes hash and the lowest uncached lane's result is inserted.
                // Exact 16-dword compare: results are unchanged either way.
                uint32_t *kc = E.s_kc;
                const bool cacheable = b.w[0] == 64u && (a.w[0] & 3u) == 0u;
                uint32_t din[16];
                bool hit = false;
                if (cacheable) {
#pragma unroll
                    for (int k = 0; k < 16; ++k) din[k] = V.mdw_safe((a.w[0] >> 2) + (uint32_t)k);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    const uint32_t valid = kc[KC_E * 24u];
                    for (uint32_t e = 0; e < KC_E; ++e) {
                        if (!((valid >> e) & 1u)) continue;
                        bool eq = true;
#pragma unroll
                        for (int k = 0; k < 16; ++k) eq = eq && kc[e * 24u + k] == din[k];
                        if (eq && !hit) {
                            hit = true;
#pragma unroll
                            for (int k = 0; k < 8; ++k) res.w[k] = kc[e * 24u + 16u + k];
                        }
                    }
                }
                const uint64_t act = __ballot(true);
                if (__ballot(hit) == act) {
                    if (L.rec_cap) {
                        uint32_t *rp = L.rec + lane + (size_t)(rec_at + MG_REC_HEADER) * L.N;
#pragma unroll
                        for (int k = 0; k < 16; ++k) rp[(size_t)k * L.N] = din[k];
                    }
                } else {
                    res = keccak_mem(V, a.w[0], b.w[0],
                                     L.rec_cap ? L.rec + lane + (size_t)(rec_at + MG_REC_HEADER) * L.N : nullptr,
                                     L.N);
                    const uint64_t ins = __ballot(cacheable && !hit);
                    if (ins != 0ull && (uint32_t)__builtin_ctzll(ins) == (threadIdx.x & 63u)) {
                        const uint32_t e = kc[KC_E * 24u + 1u] % KC_E;
#pragma unroll
                        for (int k = 0; k < 16; ++k) kc[e * 24u + k] = din[k];
#pragma unroll
                        for (int k = 0; k < 8; ++k) kc[e * 24u + 16u + k] = res.w[k];
                        kc[KC_E * 24u] = kc[KC_E * 24u] | (1u << e);
                        kc[KC_E * 24u + 1u] = e + 1u;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                }
                if (L.rec_cap) {
                    rec_head(L, lane, rec_at, MG_REC_KECCAK, b.w[0], L.steps[lane] + R.step, res);
                    rec_new = rec_at + MG_REC_HEADER + ((b.w[0] + 3u) >> 2);
                }
                if (prof) { atomicAdd(&s_prof[256], b.w[0]); atomicAdd(&s_prof[259], b.w[0] / 136u + 1u); }
            }
            ++R.n_sha3;
            break;
        }
        case K_CDLOAD: {  // byte (off+k) mod 2^256, 0 past the end (calldata.py:46-90,137-146)
            const uint32_t cdl = L.calldata_len[lane];
            const bool fits = u_fits32(a);
            if (fits && (a.w[0] & 3u) == 0u && (uint64_t)a.w[0] + 32u <= cdl) {
                const uint32_t d0 = a.w[0] >> 2;
#pragma unroll
                for (int k = 0; k < 8; ++k) res.w[7 - k] = V.cdw(d0 + k);
            } else {
                bool wrapc = true;
#pragma unroll
                for (int k = 1; k < 8; ++k) wrapc = wrapc && a.w[k] == 0xffffffffu;
                for (uint32_t k = 0; k < 32u; ++k) {
                    const uint64_t t = (uint64_t)a.w[0] + k;
                    bool ok = false;
                    uint32_t idx = 0;
                    if (fits) { ok = t < cdl; idx = (uint32_t)t; }
                    else if (wrapc && t >= (1ull << 32)) { idx = (uint32_t)(t - (1ull << 32)); ok = idx < cdl; }
                    if (ok) {
                        const uint32_t byte = V.cbyte(idx), sh = 8u * (31u - k);
                        res = u_or(res, u_shl_n(u_small(byte), sh));
                    }
                }
            }
            break;
        }
        case K_CDCOPY: {  // nothing at all for size 0 (:806-891)
            if (u_iszero(c)) break;
            MEMX(a, c, (int64_t)gtab_min)
            GASCOMMIT()
            ZEROFILL()
            const uint32_t cdl = L.calldata_len[lane];
            const bool bfits = u_fits32(b);
            bool wrapc = true;
#pragma unroll
            for (int k = 1; k < 8; ++k) wrapc = wrapc && b.w[k] == 0xffffffffu;
            if (prof) atomicAdd(&s_prof[257], c.w[0]);
            for (uint32_t k = 0; k < c.w[0]; ++k) {
                const uint64_t t = (uint64_t)b.w[0] + k;
                uint32_t v = 0u;
                if (bfits) { if (t < cdl) v = V.cbyte((uint32_t)t); }
                else if (wrapc && t >= (1ull << 32) && t - (1ull << 32) < cdl) v = V.cbyte((uint32_t)(t - (1ull << 32)));
                V.set_mbyte(a.w[0] + k, v);
            }
            break;
        }
        case K_CODECOPY: {  // extends even for size 0; copy stops at the end of code
            // creation transaction (symbolic calldata): an offset at or past the end
            // of the code copies constructor arguments (instructions.py:1089-1098)
            if ((E.flags & LANE_CREATION) && !(u_fits32(b) && b.w[0] < C.n_bytes)) ESCX(ESC_OPCODE)
            MEMX(a, c, (int64_t)gtab_min)
            GASCOMMIT()
            ZEROFILL()
            uint32_t ncopy = 0u;
            if (u_fits32(b) && b.w[0] < C.n_bytes) ncopy = min(C.n_bytes - b.w[0], c.w[0]);
            if (prof) atomicAdd(&s_prof[257], ncopy);
            for (uint32_t k = 0; k < ncopy; ++k) V.set_mbyte(a.w[0] + k, a8[C.bytes_off + b.w[0] + k]);
            break;
        }
        case K_MLOAD:
            MEMX(a, u_small(32), (int64_t)gtab_min)
            GASCOMMIT()
            ZEROFILL()
            res = V.mword(a.w[0]);
            break;
        case K_MSTORE:
            MEMX(a, u_small(32), (int64_t)gtab_min)
            GASCOMMIT()
            ZEROFILL()
            V.set_mword(a.w[0], b);
            break;
        case K_MSTORE8:
            MEMX(a, u_small(1), (int64_t)gtab_min)
            GASCOMMIT()
            ZEROFILL()
            V.set_mbyte(a.w[0], b.w[0] & 0xffu);
            break;
        case K_SLOAD: {  // over K(0) + stores (account.py:43-74)
            const uint32_t cnt = L.storage_count[lane];
            if (prof) atomicAdd(&s_prof[258], cnt);
            for (uint32_t s = 0; s < cnt; ++s) {
                const size_t base = V.row(s) * 2;
                if (u_eq(ld_word(gv(L.storage), base), a)) { res = ld_word(gv(L.storage), base + 1); break; }
            }
            break;
        }
        case K_SSTORE: {
            const uint32_t cnt = L.storage_count[lane];
            if (prof) atomicAdd(&s_prof[258], cnt);
            uint32_t slot = cnt;
            for (uint32_t s = 0; s < cnt; ++s)
                if (u_eq(ld_word(gv(L.storage), V.row(s) * 2), a)) { slot = s; break; }
            if (slot == cnt && cnt >= L.storage_cap) ESCX(ESC_STORAGE)
            GASCOMMIT()
            if (slot == cnt) {
                st_word(gv(L.storage), V.row(slot) * 2, a);
                L.storage_count[lane] = cnt + 1u;
            }
            st_word(gv(L.storage), V.row(slot) * 2 + 1, b);
            break;
        }
        case K_JUMP: {  // gas 8 by hand, no OOG check (:1520-1556)
            by_table = false;
            uint32_t idx = MG_JRES_NONE;
            if (u_fits32(a) && a.w[0] < C.n_jres) idx = a32[C.jres_off + a.w[0]];
            if (!JUMP_OK(idx)) EXCX(EXC_BADJUMP)
            ngmin += 8u; ngmax += 8u; npc = idx;
            if (FENT_AT(idx)) nfent = idx;
            break;
        }
        case K_JUMPI: {  // gas 10 by hand, depth + 1 on the side taken (:1558-1636)
            by_table = false;
            if (u_iszero(b)) {
                ngmin += 10u; ngmax += 10u; ++ndepth;
                if ((uk >> 23) & 1u) nfent = pc + 1u;      // PD_NFENT: the fall-through
            } else {
                uint32_t idx = MG_JRES_NONE;
                if (u_fits32(a) && a.w[0] < C.n_jres) idx = a32[C.jres_off + a.w[0]];
                if (!JUMP_OK(idx)) STOPX(ST_DROPPED, 0u)
                ngmin += 10u; ngmax += 10u; ++ndepth; npc = idx;
                if (FENT_AT(idx)) nfent = idx;
            }
            break;
        }
        case K_BEGINSUB: EXCX(EXC_OOG)
        case K_RETURN:  // (:1857-1874)
            MEMX(a, b, 0)
            if (ngmin >= glim) EXCX(EXC_OOG)
            L.ret_offset[lane] = a.w[0]; L.ret_len[lane] = b.w[0];
            STOPX(ST_RETURN, 0u)
        case K_REVERT:  // no memory extension (:1899-1934)
            L.ret_offset[lane] = a.w[0]; L.ret_len[lane] = b.w[0];
            STOPX(ST_REVERT, 0u)
        case K_INVALID: EXCX(EXC_INVALID)
        default: ESCX(ESC_OPCODE)
        }
        if (stop != ST_RUNNING) break;
        if (tos_done) { GASCOMMIT() break; }
        // new top-of-stack registers from the pops / push of this opcode
        if (push) {   // MachineStack.append: overflow check precedes the write
            if (nsp + 1u > STACK_LIMIT) EXCX(EXC_OVERFLOW)
            if (nsp + 1u > L.stack_cap) ESCX(ESC_STACK)
            GASCOMMIT()
            if (npop == 0u) {            // T1 moves below the register window
                if (sp >= 2u && !E.tosmem) V.set_stack(sp - 2u, b);
                R.T1 = a;
            } else if (npop >= 2u) {
                R.T1 = sp >= npop + 1u ? V.stack(sp - npop - 1u) : u_zero();
            }
            R.T0 = res;
        } else {
            GASCOMMIT()
            if (npop == 1u) {
                R.T0 = b;
                R.T1 = sp >= 3u ? V.stack(sp - 3u) : u_zero();
            } else if (npop >= 2u) {
                R.T0 = sp >= npop + 1u ? V.stack(sp - npop - 1u) : u_zero();
                R.T1 = sp >= npop + 2u ? V.stack(sp - npop - 2u) : u_zero();
            }
        }
    } while (0);
#undef STOPX
#undef EXCX
#undef ESCX
#undef GASCOMMIT
#undef MEMX
#undef ZEROFILL
#undef JUMP_OK
#undef FENT_AT
    R.stop = stop;
    R.sx = sx;
    if (stop == ST_RUNNING) {
        if (rec_new) L.rec_len[lane] = rec_new;
        R.pc = npc; R.sp = nsp + (push ? 1u : 0u);
        R.msize = nmsize; R.depth = ndepth; R.gmin = ngmin; R.gmax = ngmax; R.fent = nfent;
    }
}

// The opcodes the fast loop executes itself (when their preconditions hold).
DEV bool alu_is_fast(uint32_t op) { return op <= 0x03u || op == 0x0bu || (op >= 0x10u && op <= 0x1du); }

// Pre-decoded word (s_pd[i].y): op | req << 8 | npop << 12 | push << 16 |
// kind << 17 | PD_CREATION | PD_SPECIAL | hook << 31.
#define PD_FENT (1u << 22)       // a JUMP / JUMPI landing here switches active_function_name
#define PD_NFENT (1u << 23)      // ... landing on the next instruction (JUMPI fall-through)
#define PD_CREATION (1u << 29)   // escapes when the lane is a creation transaction
#define PD_SPECIAL (1u << 30)    // kind >= K_ESCAPE (host opcode or past-the-end)
DEV uint32_t pd_flags(uint32_t op, uint32_t dy, uint32_t hook) {
    const uint32_t kind = (dy >> 9) & 31u;
    return (hook << 31) | (kind >= K_ESCAPE ? PD_SPECIAL : 0u) | (op - 0x35u < 4u ? PD_CREATION : 0u);
}

// ---- BoundedLoopsStrategy (bounded_loops.py:49-145) ---------------------------
// The trace holds the byte address of every instruction the path was popped at.
// get_loop_count: find the latest earlier occurrence (index >= 1) of the last two
// addresses, take the segment between it and the current JUMPDEST as the key,
// and count how many consecutive copies of it end the trace, where "equal" is
// equality of calculate_hash = OR of address << 8k over the segment.  For
// 16-bit addresses byte k of that hash is lo8(S[k]) | hi8(S[k-1]), so two
// segments compare in one streaming pass.  Only called at JUMPDESTs.
__device__ __noinline__ uint32_t loop_count_dev(const uint32_t *__restrict__ T, size_t N, uint32_t n) {
    if (n < 4u) return 0u;
    const uint32_t a = T[(size_t)(n - 2u) * N], b = T[(size_t)(n - 1u) * N];
    int32_t i = (int32_t)n - 3;
    for (; i >= 1; --i)
        if (T[(size_t)i * N] == a && T[(size_t)(i + 1) * N] == b) break;
    if (i < 1) return 0u;
    const uint32_t size = n - (uint32_t)i - 2u, base = (uint32_t)i + 1u;
    uint32_t count = 2u;                    // the key segment matches itself
    for (int32_t j = (int32_t)base - (int32_t)size; j >= 0; j -= (int32_t)size) {
        uint32_t pj = 0u, pb = 0u;
        bool eq = true;
        for (uint32_t k = 0; k <= size; ++k) {
            const uint32_t xj = k < size ? T[(size_t)((uint32_t)j + k) * N] : 0u;
            const uint32_t xb = k < size ? T[(size_t)(base + k) * N] : 0u;
            if (((xj & 0xffu) | (pj >> 8)) != ((xb & 0xffu) | (pb >> 8))) { eq = false; break; }
            pj = xj;
            pb = xb;
        }
        if (!eq) break;
        ++count;
    }
    return count;
}

// Append `addr` to the lane's trace; at a JUMPDEST apply the bound.  Returns the
// new length (bits 0..31), the loop count (32..59) and the outcome (60..61):
// 0 continue, 1 dropped by the bound, 2 trace full (escape to the host).
__device__ __noinline__ uint64_t trace_step(uint32_t *__restrict__ trace, size_t N, uint32_t cap, uint32_t lane,
                                            uint32_t tlen, uint32_t addr, uint32_t jumpdest, uint32_t bound,
                                            uint32_t creation) {
    if (tlen >= cap) return (uint64_t)tlen | (2ull << 60);
    trace[(size_t)tlen * N + lane] = addr;
    ++tlen;
    if (!jumpdest) return tlen;
    const uint32_t count = loop_count_dev(trace + lane, N, tlen);
    // creation transactions only drop from max(128, bound) on (bounded_loops.py:137-145)
    const bool drop = creation ? (count > bound && count >= 128u) : count > bound;
    return (uint64_t)tlen | ((uint64_t)count << 32) | (drop ? (1ull << 60) : 0ull);
}

// ---- the stepping kernel -------------------------------------------------------
// At 65,536 lanes there is one wave per SIMD, so a wave's instruction stream is
// the bound: the loop keeps every per-step dependency on chip and dispatches
// on wave-uniform values.
//   * the block's code is pre-decoded into LDS: one 8-byte LDS read per step
//     yields opcode, gas, stack counts and handler kind;
//   * each iteration executes one opcode for the group of live lanes whose next
//     instruction decodes like the lowest live lane's, so opcode, gas and stack
//     effects are scalars and dispatch is a scalar branch;
//   * the two top stack words live in registers, the next 14 in an LDS window,
//     the rest in HBM;
//   * common opcodes run inline; the rest (and any lane whose preconditions
//     fail) go through slow_step, inlined too: the kernel uses no scratch.
// kLoop: BoundedLoopsStrategy traces on (a separate instantiation, so the common
// case carries no trace call site in its loop)
// Re-initialise one lane from the resident image (mg_lanes_reset): empty stack,
// memory, traces and record logs; pc, depth, status, gas and storage from the image.
__device__ __forceinline__ void reset_lane(const DevLanes &L, const DevResetImage &R, uint32_t lane) {
    L.pc[lane] = R.pc[lane]; L.sp[lane] = 0; L.msize[lane] = 0; L.depth[lane] = R.depth[lane];
    L.status[lane] = R.status[lane]; L.aux[lane] = R.aux[lane]; L.steps[lane] = R.steps[lane];
    L.gas_min[lane] = R.gas_min[lane]; L.gas_max[lane] = R.gas_max[lane];
    L.sha3_count[lane] = 0; L.exp_count[lane] = 0;
    L.trace_len[lane] = 0;                 // reset images start with empty traces
    L.rec_len[lane] = 0;                   // ... and empty record logs
    L.fent[lane] = MG_FENT_NONE;           // ... and no function switch yet
    const uint32_t cnt = R.storage_count[lane];
    L.storage_count[lane] = cnt;
    for (uint32_t s = 0; s < cnt; ++s)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const size_t idx = ((size_t)s * L.N + lane) * 4 + k;
            L.storage[idx] = R.storage[idx];
        }
}

#ifdef MG_K1_CLOCKS
// Diagnostic build only (scripts/k1_clocks.py): shader-clock cycles per wave,
// binned by the opcode each dispatch-loop iteration executed (bin 256: a
// straight-line run, 257: prologue, 258: epilogue, 259: iterations that
// advanced no lane of this wave).  Lane 0 of each wave keeps its bins in LDS
// and writes them out with plain vector stores at the end.  Each bin packs
// cycles in bits 0-23 and the number of iterations in bits 24-31.
#define CLK_BINS 262u   // opcode bins, 256 runs, 257 prologue, 258 epilogue, 259 idle,
                        // 260 dispatch head (loop top -> decoded), 261 FETCH of the next pc
__device__ uint32_t g_k1_clk[4096u * CLK_BINS];
#endif

template <bool kLoop>
__global__ __launch_bounds__(LANE_BLOCK) void k_lane_step(DevLanes L, const DevCode *__restrict__ codes,
                                                          const uint8_t *__restrict__ a8,
                                                          const uint32_t *__restrict__ a32,
                                                          uint8_t *__restrict__ cov, uint32_t cov_on,
                                                          uint64_t m0, uint64_t m1, uint64_t m2, uint64_t m3,
                                                          uint32_t max_steps, uint32_t max_depth,
                                                          DevCounters *__restrict__ ctr,
                                                          unsigned long long *__restrict__ prof,
                                                          uint32_t win, uint32_t pd_cap, uint32_t jr_cap,
                                                          uint32_t horizon, uint32_t loop_bound,
                                                          DevResetImage R, uint32_t lpw_flags) {
    // lpw_flags: lanes per wave in bits 0..7; bit 8 = register-form runs only
    // (MG_K1_RUNS=reg, for A/B runs against the LDS-resident form); bit 9 = the
    // push immediates are staged in LDS too (otherwise read from the code arena
    // at wave-uniform addresses)
    const uint32_t lpw = lpw_flags & 0xffu;
    const bool lds_runs_on = (lpw_flags & 0x100u) == 0u;
    const bool push_lds = (lpw_flags & 0x200u) != 0u;
    // bits 16..23: LDS memory window per lane in 32-byte words
    const uint32_t mw = ((lpw_flags >> 16) & 0xffu) * 8u;
    // Dynamic LDS: [stack window: win x 2 x lanes-per-block x 16 B]
    //              [memory window: mw x lanes-per-block x 4 B]
    //              [pre-decoded code: pd_cap x 16 B: decode x, y | run table z, w]
    //              [push immediates: pd_cap x 32 B, when push_lds][jump-resolve: jr_cap x 2 B]
    //              [coverage: pd_cap]
    // A code longer than pd_cap - 1 instructions is staged as its first
    // pd_cap - 1 instructions (and its first jr_cap jump targets); the lanes
    // beyond that prefix decode from the code arena and run no straight-line runs.
    // One ds_read_b128 at FETCH brings a lane both its next instruction's decode
    // and the straight-line run starting there, so the dispatch head reads the
    // lead lane's run with v_readlane instead of another dependent LDS read.
    extern __shared__ __attribute__((aligned(16))) uint4 dyn[];
    l_u4 *s_win = (l_u4 *)dyn;
    // Lanes per wave (`lpw` = 64, 32 or 16, launch-uniform): each wave holds lpw
    // lanes in its first lpw threads and the rest idle, so a launch of n lanes has
    // n / lpw waves.  At C2's 65,536 lanes, lpw = 64 is one wave per SIMD and the
    // launch is bound by one wave's serial dispatch chain; fewer lanes per wave
    // put 2 or 4 waves on each SIMD, whose chains then overlap (and each wave's
    // lanes diverge less).  The idle threads still take part in the wave-wide
    // LDS load of a run's pre-decoded words below.
    const uint32_t lanes_pb = (LANE_BLOCK / 64u) * lpw;
    l_u32 *s_mw = (l_u32 *)(dyn + (size_t)win * 2u * lanes_pb);
    uint4 *s_pd = dyn + (size_t)win * 2u * lanes_pb + (size_t)mw * lanes_pb / 4u;
    uint4 *s_push = s_pd + pd_cap;
    uint16_t *s_jr = reinterpret_cast<uint16_t *>(s_push + (push_lds ? 2u * pd_cap : 0u));
    uint8_t *s_cov = reinterpret_cast<uint8_t *>(s_jr + jr_cap);
    __shared__ uint2 s_dec[256];
    __shared__ uint32_t s_code;
    // optional instruction profile (InstructionProfiler's per-opcode counts,
    // instruction_profiler.py:41-115, as native counters): 256 opcode counts +
    // [sha3 bytes, copy bytes, storage entries scanned, keccak blocks]
    __shared__ uint32_t s_prof[260];
    __shared__ uint32_t s_kc[(LANE_BLOCK / 64u) * KC_WAVE];

    const uint32_t wlane = threadIdx.x & 63u;
    const uint32_t tid = (threadIdx.x >> 6) * lpw + wlane;     // lane index in the block
    const uint32_t lane = blockIdx.x * lanes_pb + tid;
    const bool in_range = wlane < lpw && lane < L.n;
    // mg_run_batches: re-initialise the lane from the resident image first (the
    // reads below see this thread's own stores)
    if (R.pc != nullptr && in_range) reset_lane(L, R, lane);
    uint32_t status = in_range ? L.status[lane] : ST_STOP;
    const uint32_t my_code = in_range ? L.code_id[lane] : 0u;
    for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) s_dec[i] = kDec[i];
    if (prof)
        for (uint32_t i = threadIdx.x; i < 260u; i += blockDim.x) s_prof[i] = 0u;
    if (threadIdx.x == 0) s_code = 0xffffffffu;
    if ((threadIdx.x & 63u) < 2u) s_kc[(threadIdx.x >> 6) * KC_WAVE + KC_E * 24u + (threadIdx.x & 63u)] = 0u;
    __syncthreads();
    if (status == ST_RUNNING) s_code = my_code;      // any running lane's code (benign race)
    __syncthreads();
#ifdef MG_K1_CLOCKS
    __shared__ uint32_t s_clk[LANE_BLOCK / 64u][CLK_BINS];
    for (uint32_t i = threadIdx.x; i < (LANE_BLOCK / 64u) * CLK_BINS; i += blockDim.x) (&s_clk[0][0])[i] = 0u;
    __syncthreads();
    // wave-uniform clock state in LDS, updated by the first active lane, so a
    // mark inside a divergent region charges the right bin
    __shared__ uint64_t s_clk_t[LANE_BLOCK / 64u];
    __shared__ uint32_t s_clk_bin[LANE_BLOCK / 64u];
    if ((threadIdx.x & 63u) == 0u) { s_clk_t[threadIdx.x >> 6] = __builtin_amdgcn_s_memtime();
                                     s_clk_bin[threadIdx.x >> 6] = 257u; }
#define CLK_MARK(next_) do { const uint64_t t_ = __builtin_amdgcn_s_memtime();                   \
        const uint64_t act_ = __ballot(1);                                                     \
        if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(act_)) {                           \
            const uint32_t w_ = threadIdx.x >> 6;                                              \
            s_clk[w_][s_clk_bin[w_]] += (uint32_t)(t_ - s_clk_t[w_]) + (1u << 24);             \
            s_clk_t[w_] = t_; s_clk_bin[w_] = (next_); } } while (0)
#else
#define CLK_MARK(next_) do { } while (0)
#endif
    const uint32_t bcode = s_code;
    const bool mixed = __syncthreads_or(status == ST_RUNNING && my_code != bcode);
    bool staged = false, jstaged = false;
    uint32_t ns_b = 0u, sn_b = 0u, jn_b = 0u, push_b = 0u;
    if (bcode != 0xffffffffu && !mixed) {
        const DevCode BC = codes[bcode];
        const uint32_t ns = min(BC.n_instr, pd_cap - 1u);   // staged prefix
        if (ns > 0u) {
            // pre-decode: opcode, gas, stack counts, kind, and the hook bit (bit 31)
            for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
                const uint32_t op = a8[BC.op_off + i];
                const uint2 d = kDec[op];
                const uint64_t hm = op < 64u ? m0 : op < 128u ? m1 : op < 192u ? m2 : m3;
                const uint32_t hook = (uint32_t)((hm >> (op & 63u)) & 1ull);
                s_pd[i] = make_uint4(d.x, op | (d.y << 8) | pd_flags(op, d.y, hook) |
                                              ((uint32_t)a8[BC.fent_off + i] << 22),
                                     a32[BC.run_off + 2u * i], a32[BC.run_off + 2u * i + 1u]);
                s_cov[i] = 0;
            }
            if (threadIdx.x == 0 && ns == BC.n_instr)
                s_pd[ns] = make_uint4(0u, ((uint32_t)K_END << 17) | PD_SPECIAL, 0u, 0u);
            if (push_lds) {        // the host plans push_lds only for wholly staged codes
                const uint4 *gpu4 = reinterpret_cast<const uint4 *>(a32 + BC.push_off);
                for (uint32_t i = threadIdx.x; i < 2u * ns; i += blockDim.x) s_push[i] = gpu4[i];
            }
            staged = true;
            ns_b = ns;
            sn_b = ns == BC.n_instr ? ns + 1u : ns;
            push_b = BC.push_off;
            const uint32_t jn = min(BC.n_jres, jr_cap);
            if (jn > 0u && BC.n_instr < 0xffffu) {
                for (uint32_t i = threadIdx.x; i < jn; i += blockDim.x) {
                    const uint32_t t = a32[BC.jres_off + i];
                    s_jr[i] = t == MG_JRES_NONE ? (uint16_t)0xffffu : (uint16_t)t;
                }
                jstaged = true;
                jn_b = jn;
            }
        }
        __syncthreads();
    }
    uint32_t executed = 0;
    // symbolic and taint lanes (MG_LANE_SYMBOLIC, MG_LANE_TAINT) are k_sym_step's: counted as running, untouched
    const bool sym_lane = in_range && status == ST_RUNNING && (L.flags[lane] & (16u | 2048u)) != 0u;
    const bool run0 = status == ST_RUNNING && !sym_lane;
    // block-uniform facts in scalar registers
    const uint32_t sflag = __builtin_amdgcn_readfirstlane(staged ? 1u : 0u);
    const uint32_t jflag = __builtin_amdgcn_readfirstlane(jstaged ? 1u : 0u);
    const uint32_t ns = __builtin_amdgcn_readfirstlane(ns_b);     // staged instructions
    const uint32_t sn = __builtin_amdgcn_readfirstlane(sn_b);     // + the END sentinel
    const uint32_t jn = __builtin_amdgcn_readfirstlane(jn_b);     // staged jump targets
    const uint32_t bpush = __builtin_amdgcn_readfirstlane(push_b);
    const uint32_t psflag = (staged && push_lds) ? 1u : 0u;
    // push immediate of instruction i of the staged code (wave-uniform i in runs)
#define PUSH_IMM(i_) (psflag ? ld_word((const l_u4 *)s_push, (i_)) : ld_word(gv(a32 + bpush), (i_)))
    const uint32_t stack_lim = L.stack_cap < STACK_LIMIT ? L.stack_cap : STACK_LIMIT;

    // ---- per-lane machine state (registers) ----
    const LaneView V{L, lane, s_win, win, tid, lanes_pb, s_mw, mw};
    DevCode C{};
    uint32_t flags = 0, pc = 0, sp = 0, msize = 0, depth = 0, aux = 0, n_sha3 = 0, n_exp = 0;
    uint32_t tlen = 0;                                    // trace length (BoundedLoops)
    uint32_t fent = MG_FENT_NONE;                         // last function-entry landing
    const uint32_t loop_on = kLoop ? loop_bound : 0u;     // kernel argument: uniform
    uint64_t txlim = 0, glim = 0, gmin = 0, gmax = 0;
    U256 T0 = u_zero(), T1 = u_zero();
    uint2 pd = make_uint2(0u, 0u);
    uint2 prun = make_uint2(0u, 0u);   // run table entry at pc (staged code only)
    bool live = false;
    if (run0) {
        C = codes[my_code];
        flags = L.flags[lane];
        txlim = L.gas_limit[lane];
        // accumulate_gas OOG test (instructions.py:162-176): min > 1e9 or min >= tx gas limit
        glim = txlim < MSTATE_GAS_LIMIT + 1ull ? txlim : MSTATE_GAS_LIMIT + 1ull;
        pc = L.pc[lane]; sp = L.sp[lane]; msize = L.msize[lane]; depth = L.depth[lane];
        fent = L.fent[lane];
        if (loop_on) tlen = L.trace_len[lane];
        gmin = L.gas_min[lane]; gmax = L.gas_max[lane];
        for (uint32_t k = 0; k < min(sp, win); ++k) V.set_wstack(k, V.gstack(k));   // window fill
        for (uint32_t k = 0; k < min(msize >> 2, mw); ++k) V.set_lmdw(k, V.gmdw(k));
        if (sp >= 1u) T0 = V.stack(sp - 1u);
        if (sp >= 2u) T1 = V.stack(sp - 2u);
        live = true;
    }
    const bool creation = (flags & LANE_CREATION) != 0u;
    // host hook protocol: HOOK_ACK lets the first instruction of this call run past
    // its hook bit; STEP1 caps the lane at one instruction (post-hooks)
    const bool hook_ack = (flags & LANE_HOOK_ACK) != 0u;
    uint32_t lane_max = (flags & LANE_STEP1) ? min(max_steps, 1u) : max_steps;
    // step horizon (mg_step_until): the lane pauses once its cumulative steps reach it
    if (horizon && run0) {
        const uint32_t s0 = L.steps[lane];
        lane_max = min(lane_max, horizon > s0 ? horizon - s0 : 0u);
    }
    const uint8_t *__restrict__ gops = a8 + C.op_off;
    const uint8_t *__restrict__ gfent = a8 + C.fent_off;
    const StepEnv E{&L, C, a8, a32, s_win, s_mw, s_pd, s_push, s_prof, s_kc + (threadIdx.x >> 6) * KC_WAVE,
                    txlim, glim, lane, tid, lanes_pb, win, flags, sflag, psflag, prof ? 1u : 0u, mw, sn, 0u};

    // Decode the instruction at pc and run the checks svm.execute_state makes
    // before evaluating it (svm.py:369-402): depth cut-off, past-the-end pc,
    // hooked opcode, this launch's step budget, host-only opcode.
#define FETCH() do { FETCH_LOAD(); FETCH_CHECK(); } while (0)
    // MG_K1_PF (A/B builds): the single-instruction path loads the entry of pc + 1
    // before its handler runs and FETCH_PF uses it when the lane fell through
#define FETCH_PF(q_pf, pc_pf) do {                                                        \
        if (sflag && pc == (pc_pf) && pc < sn) {                                          \
            pd = make_uint2((q_pf).x, (q_pf).y); prun = make_uint2((q_pf).z, (q_pf).w);   \
        } else FETCH_LOAD();                                                              \
        FETCH_CHECK();                                                                    \
    } while (0)
#define FETCH_LOAD() do {                                                                 \
        if (sflag && pc < sn) {                                                           \
            const uint4 q_ = s_pd[pc];        /* s_pd[n_instr] is the END sentinel */     \
            pd = make_uint2(q_.x, q_.y); prun = make_uint2(q_.z, q_.w);                   \
        } else if (pc >= C.n_instr) {                                                     \
            pd = make_uint2(0u, ((uint32_t)K_END << 17) | PD_SPECIAL);                    \
            prun = make_uint2(0u, 0u);                                                    \
        } else {                                                                          \
            prun = make_uint2(0u, 0u);        /* no runs beyond the staged prefix */      \
            const uint32_t o_ = gops[pc];                                                 \
            const uint2 d_ = s_dec[o_];                                                   \
            const uint64_t hm_ = o_ < 64u ? m0 : o_ < 128u ? m1 : o_ < 192u ? m2 : m3;    \
            pd = make_uint2(d_.x, o_ | (d_.y << 8) | ((uint32_t)gfent[pc] << 22) |         \
                            pd_flags(o_, d_.y, (uint32_t)((hm_ >> (o_ & 63u)) & 1ull)));  \
        }                                                                                 \
    } while (0)
#define FETCH_CHECK() do {                                                                \
        const uint32_t k_ = (pd.y >> 17) & 31u, o_ = pd.y & 0xffu;                       \
        const bool hk_ = (pd.y >> 31) && !(hook_ack && executed == 0u);                  \
        bool lstop_ = false;                                                              \
        /* BoundedLoopsStrategy: every instruction the path is popped at (run,   */      \
        /* hooked or escaped; not a budget pause, not the ACK re-fetch) is traced */     \
        if (loop_on && k_ != K_END && !(max_depth != 0u && depth >= max_depth) &&        \
            !(hook_ack && executed == 0u) && (hk_ || executed < lane_max)) {              \
            const uint64_t tr_ = trace_step(L.trace, L.N, L.trace_cap, lane, tlen,        \
                                            a32[C.addr_off + pc], o_ == 0x5bu, loop_bound,\
                                            creation ? 1u : 0u);                          \
            tlen = (uint32_t)tr_;                                                         \
            const uint32_t res_ = (uint32_t)(tr_ >> 60);                                  \
            if (res_ == 1u) { status = ST_LOOP; aux = (uint32_t)(tr_ >> 32) & 0x0fffffffu; \
                              live = false; lstop_ = true; }                              \
            else if (res_ == 2u) { status = ST_ESCAPE; aux = o_ | (ESC_TRACE << 8);        \
                                   live = false; lstop_ = true; }                         \
        }                                                                                 \
        /* one test for the common case: bits 29/30 pre-decode "escape or END"  */      \
        /* and "escapes in a creation transaction" (CALLDATA*, CODESIZE/COPY)    */      \
        if (!lstop_ && (hk_ || (pd.y & PD_SPECIAL) || executed >= lane_max ||             \
            (max_depth != 0u && depth >= max_depth) || (creation && (pd.y & PD_CREATION)))) { \
            uint32_t st_ = ST_RUNNING;                                                    \
            if (max_depth != 0u && depth >= max_depth) st_ = ST_DEPTH;                    \
            else if (k_ == K_END) st_ = ST_END;                                           \
            else if (hk_) { st_ = ST_HOOK; aux = o_; }                                    \
            else if (executed >= lane_max) live = false;                                  \
            else { st_ = ST_ESCAPE; aux = o_ | (ESC_OPCODE << 8); }                       \
            if (st_ != ST_RUNNING) { status = st_; live = false; }                        \
        }                                                                                 \
    } while (0)

    if (live) FETCH();

    // Straight-line runs: with no hook, no loop bound and no profiling in this
    // launch, the lanes sitting at the lead lane's pc whose whole run passes its
    // checks at once (stack depth, stack growth, table gas, step budget) execute
    // the run as a block: one dispatch per run instead of per instruction.
    const bool runs_on = sflag && !prof && !loop_on && ((m0 | m1 | m2 | m3) == 0ull);

    for (;;) {
        CLK_MARK(260u);
        const uint64_t live_mask = __ballot(live);
        if (live_mask == 0ull) break;
        const int lead = __builtin_ctzll(live_mask);
        if (runs_on) {
            uint32_t upc = __builtin_amdgcn_readlane(pc, lead);
            asm volatile("" : "+s"(upc));
            // the lead's run entry came with its FETCH (prun): no LDS round trip here
            const uint32_t rx = __builtin_amdgcn_readlane(prun.x, lead);
            const uint32_t ry = __builtin_amdgcn_readlane(prun.y, lead);
            const uint32_t rlen = rx & 0xffu;
            if (rlen >= 2u && upc + rlen <= ns) {
                const uint32_t rneed = (rx >> 8) & 0xffu, rpeak = (rx >> 16) & 0xffu;
                // a run may end with a JUMP (rjk 1) or JUMPI (2): rsimple plain steps first
                const uint32_t rjk = (rx >> 24) & 3u, rsimple = rjk ? rlen - 1u : rlen;
                const uint32_t rg0 = ry & 0xffffu, rg1 = ry >> 16;
                // LDS-resident form: when the lead lane's whole run stays inside the
                // LDS stack window, the lanes at the lead's pc AND stack depth run it
                // with the depth as a scalar: every stack word lives in the window
                // for the run's duration (T0/T1 spilled on entry, reloaded on exit),
                // PUSH/DUP/SWAP are LDS copies at scalar offsets and POP/JUMPDEST
                // cost nothing.  Otherwise the register form below.
                uint32_t usp = __builtin_amdgcn_readlane(sp, lead);
                asm volatile("" : "+s"(usp));
                const bool lds_run = lds_runs_on && usp >= rneed && usp + rpeak <= win &&
                                     usp + rpeak <= stack_lim;
                const bool in_run = live && pc == upc && sp >= rneed && sp + rpeak <= stack_lim &&
                                    gmin + rg0 < glim && executed + rlen <= lane_max &&
                                    (!lds_run || sp == usp);
                // the run's pre-decoded words, one per wave lane (rlen <= RUN_MAX = 64),
                // read by the whole wave in one LDS access; instruction k is then
                // v_readlane(k) instead of a dependent LDS round trip per instruction
                // (opaque barrier: the load must run here with the whole wave active,
                // not be sunk into the `in_run` branch where only some lanes load)
                uint32_t ybulk = s_pd[min(upc + (threadIdx.x & 63u), pd_cap - 1u)].y;
                asm volatile("" : "+v"(ybulk));
                if ((__ballot(in_run) >> lead) & 1ull) {
                    CLK_MARK(256u);
                    if (in_run && lds_run) {
                        uint32_t s = usp;
                        if (s >= 1u) V.set_wstack(s - 1u, T0);
                        if (s >= 2u) V.set_wstack(s - 2u, T1);
                        for (uint32_t k = 0; k < rsimple; ++k) {
                            const uint32_t y = __builtin_amdgcn_readlane(ybulk, k);
                            const uint32_t rop = y & 0xffu;
                            switch ((y >> 17) & 31u) {
                            case K_PUSH:
                                V.set_wstack(s, PUSH_IMM(upc + k));
                                ++s;
                                break;
                            case K_DUP:
                                V.set_wstack(s, V.wstack(s - (rop - 0x7fu)));
                                ++s;
                                break;
                            case K_SWAP: {
                                const uint32_t d = rop - 0x8fu;
                                const U256 x = V.wstack(s - 1u), z = V.wstack(s - 1u - d);
                                V.set_wstack(s - 1u, z);
                                V.set_wstack(s - 1u - d, x);
                                break;
                            }
                            case K_POP:
                                --s;
                                break;
                            case K_ALU: {
                                const U256 a = V.wstack(s - 1u);
                                if (rop == 0x15u || rop == 0x19u) {        // ISZERO, NOT
                                    V.set_wstack(s - 1u, alu(rop, a, a, a));
                                } else {                                  // pop 2, push 1
                                    const U256 b = V.wstack(s - 2u);
                                    V.set_wstack(s - 2u, alu(rop, a, b, b));
                                    --s;
                                }
                                break;
                            }
                            default:                                      // JUMPDEST
                                break;
                            }
                        }
                        // the closing jump (instructions.py:1520-1636), per lane: a lane
                        // whose jump would raise or drop its path stops AT the jump and
                        // the single-instruction path runs it (exceptions, drops)
                        uint32_t nsp = s, npc = upc + rsimple, nexec = executed + rsimple;
                        uint32_t jg = 0u;
                        if (rjk) {
                            const U256 tgt = V.wstack(s - 1u);
                            const bool take = rjk == 1u || !u_iszero(V.wstack(s - 2u));
                            uint32_t idx = MG_JRES_NONE;
                            if (take && u_fits32(tgt) && tgt.w[0] < C.n_jres) {
                                if (jflag && tgt.w[0] < jn) { idx = s_jr[tgt.w[0]]; if (idx == 0xffffu) idx = MG_JRES_NONE; }
                                else idx = a32[C.jres_off + tgt.w[0]];
                            }
                            const uint32_t ty = take && idx != MG_JRES_NONE
                                                    ? (idx < sn ? s_pd[idx].y : (uint32_t)gops[idx] |
                                                                                ((uint32_t)gfent[idx] << 22))
                                                    : 0u;
                            if (!take || (idx != MG_JRES_NONE && (ty & 0xffu) == 0x5bu)) {
                                nsp = s - rjk;
                                npc = take ? idx : upc + rlen;
                                nexec = executed + rlen;
                                jg = rjk == 1u ? 8u : 10u;      // added by hand, no OOG check
                                if (rjk == 2u) ++depth;
                                // _new_node_state: the successor at a function entry (the
                                // fall-through's bit rides on the JUMPI's own decode word)
                                const uint32_t jy = __builtin_amdgcn_readlane(ybulk, rsimple);
                                if (take ? (ty & PD_FENT) : (jy & PD_NFENT)) fent = npc;
                            }
                        }
                        T0 = nsp >= 1u ? V.wstack(nsp - 1u) : u_zero();
                        T1 = nsp >= 2u ? V.wstack(nsp - 2u) : u_zero();
                        sp = nsp;
                        pc = npc; gmin += rg0 + jg; gmax += rg1 + jg; executed = nexec;
                        FETCH();
                    } else if (in_run) {
                        // register form: the plain steps only; a closing jump runs as
                        // its own dispatch
                        for (uint32_t k = 0; k < rsimple; ++k) {
                            const uint32_t y = __builtin_amdgcn_readlane(ybulk, k);
                            const uint32_t rop = y & 0xffu;
                            switch ((y >> 17) & 31u) {
                            case K_PUSH: {
                                const U256 v = PUSH_IMM(upc + k);
                                if (sp >= 2u) V.set_stack(sp - 2u, T1);
                                T1 = T0; T0 = v; ++sp;
                                break;
                            }
                            case K_DUP: {
                                const uint32_t d = rop - 0x7fu;
                                const U256 v = d == 1u ? T0 : d == 2u ? T1 : V.stack(sp - d);
                                if (sp >= 2u) V.set_stack(sp - 2u, T1);
                                T1 = T0; T0 = v; ++sp;
                                break;
                            }
                            case K_SWAP: {
                                const uint32_t d = rop - 0x8fu;
                                if (d == 1u) {
                                    const U256 t = T0; T0 = T1; T1 = t;
                                } else {
                                    const U256 x = V.stack(sp - 1u - d);
                                    V.set_stack(sp - 1u - d, T0);
                                    T0 = x;
                                }
                                break;
                            }
                            case K_POP:
                                T0 = T1;
                                T1 = sp >= 3u ? V.stack(sp - 3u) : u_zero();
                                --sp;
                                break;
                            case K_ALU: {
                                const U256 r = alu(rop, T0, T1, T1);
                                T0 = r;
                                if (rop != 0x15u && rop != 0x19u) {     // binary: pop 2, push 1
                                    T1 = sp >= 3u ? V.stack(sp - 3u) : u_zero();
                                    --sp;
                                }
                                break;
                            }
                            default:                                    // JUMPDEST
                                break;
                            }
                        }
                        pc = upc + rsimple; gmin += rg0; gmax += rg1; executed += rsimple;
                        FETCH();
                    }
                    if (cov_on) {
                        const uint32_t wl = threadIdx.x & 63u;
                        if (wl < rlen) s_cov[upc + wl] = 1;
                    }
                    continue;
                }
            }
        }
        const uint32_t uy = __builtin_amdgcn_readlane(pd.y, lead);
        uint32_t ux = __builtin_amdgcn_readlane(pd.x, lead), uk = uy;
        // opaque scalar copies: keep the decode below on SGPRs (otherwise the
        // compiler substitutes the per-lane pd.y, equal inside the branch)
        asm volatile("" : "+s"(uk), "+s"(ux));
        if (!(live && pd.y == uy)) continue;

        const uint32_t op = uk & 0xffu, kind = (uk >> 17) & 31u;
#if MG_K1_PF
        const uint32_t pc_pf = pc + 1u;
        const uint4 q_pf = s_pd[min(pc_pf, sn - 1u)];
#endif
        CLK_MARK(op);
        if (cov_on) {
            if (sflag && pc < ns) s_cov[pc] = 1;
            else cov[C.cov_off + pc] = 1;
        }
        if (prof) atomicAdd(&s_prof[op], 1u);
        ++executed;

        // ---- fast path: every case checks its preconditions per lane and, when
        // they hold, applies the whole instruction itself; a lane whose checks
        // fail (and every other opcode) runs the general handler below ----
        const uint64_t ngmin = gmin + (ux & 0xffffu), ngmax = gmax + (ux >> 16);
        const bool gas_ok = ngmin < glim;
        bool ok = false;
        // push `v` (table gas): T1 moves below the register window
#define PUSHV(v_) do { const U256 pv_ = (v_);                                   \
            if (sp >= 2u) V.set_stack(sp - 2u, T1);                          \
            T1 = T0; T0 = pv_; ++sp; ++pc; gmin = ngmin; gmax = ngmax; } while (0)
        switch (kind) {
        case K_PUSH:
            ok = gas_ok && sp + 1u <= stack_lim;
            if (ok) PUSHV(psflag ? ld_word((const l_u4 *)s_push, pc) : ld_word(gv(a32 + C.push_off), pc));
            break;
        case K_DUP: {
            const uint32_t k = op - 0x7fu;
            ok = gas_ok && sp >= k && sp + 1u <= stack_lim;
            if (ok) PUSHV(k == 1u ? T0 : k == 2u ? T1 : V.stack(sp - k));
            break;
        }
        case K_SWAP: {
            const uint32_t k = op - 0x8fu;
            ok = gas_ok && sp >= k + 1u;
            if (ok) {
                if (k == 1u) {
                    const U256 t = T0; T0 = T1; T1 = t;
                } else {
                    const U256 x = V.stack(sp - 1u - k);
                    V.set_stack(sp - 1u - k, T0);
                    T0 = x;
                }
                ++pc; gmin = ngmin; gmax = ngmax;
            }
            break;
        }
        case K_POP:
            ok = gas_ok && sp >= 1u;
            if (ok) {
                T0 = T1;
                T1 = sp >= 3u ? V.stack(sp - 3u) : u_zero();
                --sp; ++pc; gmin = ngmin; gmax = ngmax;
            }
            break;
        case K_JUMPDEST:
            ok = gas_ok;
            if (ok) { ++pc; gmin = ngmin; gmax = ngmax; }
            break;
        case K_JUMP: case K_JUMPI: {   // gas 8 / 10 by hand, no OOG check
            const bool jumpi = kind == K_JUMPI;
            const bool take = !jumpi || !u_iszero(T1);
            uint32_t npc = pc + 1u;
            uint32_t fbit = uk & PD_NFENT;              // the fall-through's entry bit
            ok = sp >= (jumpi ? 2u : 1u);
            if (take) {
                uint32_t idx = MG_JRES_NONE;
                if (u_fits32(T0) && T0.w[0] < C.n_jres) {
                    if (jflag && T0.w[0] < jn) { idx = s_jr[T0.w[0]]; if (idx == 0xffffu) idx = MG_JRES_NONE; }
                    else idx = a32[C.jres_off + T0.w[0]];
                }
                const uint32_t ty = idx != MG_JRES_NONE
                                        ? ((sflag && idx < sn) ? s_pd[idx].y
                                                               : (uint32_t)gops[idx] | ((uint32_t)gfent[idx] << 22))
                                        : 0u;
                ok = ok && idx != MG_JRES_NONE && (ty & 0xffu) == 0x5bu;
                npc = idx;
                fbit = ty & PD_FENT;
            }
            if (ok) {
                const uint32_t add = jumpi ? 10u : 8u;
                if (fbit) fent = npc;                   // _new_node_state (svm.py:617-637)
                gmin += add; gmax += add;
                if (jumpi) {
                    ++depth;
                    T0 = sp >= 3u ? V.stack(sp - 3u) : u_zero();
                    T1 = sp >= 4u ? V.stack(sp - 4u) : u_zero();
                    sp -= 2u;
                } else {
                    T0 = T1;
                    T1 = sp >= 3u ? V.stack(sp - 3u) : u_zero();
                    --sp;
                }
                pc = npc;
            }
            break;
        }
        case K_ALU:
            if (alu_is_fast(op)) {
                const bool unary = op == 0x15u || op == 0x19u;      // ISZERO, NOT
                ok = gas_ok && sp >= (unary ? 1u : 2u);
                if (ok) {
                    const U256 r = alu(op, T0, T1, T1);
                    if (unary) {
                        T0 = r;
                    } else {
                        T0 = r;
                        T1 = sp >= 3u ? V.stack(sp - 3u) : u_zero();
                        --sp;
                    }
                    ++pc; gmin = ngmin; gmax = ngmax;
                }
            }
            break;
        case K_ENV:
            ok = gas_ok && sp + 1u <= stack_lim && !(op == 0x3du && (flags & LANE_RETDATA));
            if (ok) {
                U256 r;
                switch (op) {
                case 0x30: r = V.env(0); break;                 // ADDRESS
                case 0x32: r = V.env(2); break;                 // ORIGIN
                case 0x33: r = V.env(1); break;                 // CALLER
                case 0x34: r = V.env(3); break;                 // CALLVALUE
                case 0x3a: r = V.env(4); break;                 // GASPRICE
                case 0x36: r = u_small(L.calldata_len[lane]); break;
                case 0x38: r = u_small(C.n_bytes); break;       // CODESIZE
                case 0x45: r = u_small(MSTATE_GAS_LIMIT); break;
                case 0x58: r = u_small(a32[C.addr_off + pc]); break;
                case 0x59: r = u_small(msize); break;
                default: r = u_zero(); break;                   // RETURNDATASIZE
                }
                PUSHV(r);
            }
            break;
        case K_MLOAD:                   // inside msize: no extension, table gas only
            ok = gas_ok && sp >= 1u && u_fits32(T0) && msize >= 32u && T0.w[0] <= msize - 32u;
            if (ok) { T0 = V.mword(T0.w[0]); ++pc; gmin = ngmin; gmax = ngmax; }
            break;
        case K_MSTORE:
            ok = gas_ok && sp >= 2u && u_fits32(T0) && msize >= 32u && T0.w[0] <= msize - 32u;
            if (ok) {
                V.set_mword(T0.w[0], T1);
                T0 = sp >= 3u ? V.stack(sp - 3u) : u_zero();
                T1 = sp >= 4u ? V.stack(sp - 4u) : u_zero();
                sp -= 2u; ++pc; gmin = ngmin; gmax = ngmax;
            }
            break;
        case K_CDLOAD: {                // aligned and inside the calldata
            const uint32_t cdl = L.calldata_len[lane];
            ok = gas_ok && sp >= 1u && u_fits32(T0) && (T0.w[0] & 3u) == 0u &&
                 (uint64_t)T0.w[0] + 32u <= cdl;
            if (ok) {
                const uint32_t d0 = T0.w[0] >> 2;
                U256 r;
#pragma unroll
                for (int k = 0; k < 8; ++k) r.w[7 - k] = V.cdw(d0 + k);
                T0 = r; ++pc; gmin = ngmin; gmax = ngmax;
            }
            break;
        }
        default:
            break;
        }
#undef PUSHV
        if (!ok) {
            LaneRegs R{T0, T1, gmin, gmax, pc, sp, msize, depth, n_sha3, n_exp, 0u, 0u, executed - 1u, fent};
            slow_step(R, E, uk, ux);
            n_sha3 = R.n_sha3; n_exp = R.n_exp;
            if (R.stop != ST_RUNNING) {
                status = R.stop;
                aux = R.sx;
                if (R.stop == ST_ESCAPE) --executed;
                live = false;
            } else {
                T0 = R.T0; T1 = R.T1; gmin = R.gmin; gmax = R.gmax;
                pc = R.pc; sp = R.sp; msize = R.msize; depth = R.depth; fent = R.fent;
            }
        }
        CLK_MARK(261u);
#if MG_K1_PF
        if (live) FETCH_PF(q_pf, pc_pf);
#else
        if (live) FETCH();
#endif
    }
#undef FETCH_PF
#undef FETCH_LOAD
#undef FETCH_CHECK
#undef FETCH
#undef PUSH_IMM
    CLK_MARK(258u);

    if (run0) {
        // flush the registers, then the LDS window: HBM holds the canonical S[0 .. sp)
        if (sp >= 1u) V.set_stack(sp - 1u, T0);
        if (sp >= 2u) V.set_stack(sp - 2u, T1);
        for (uint32_t k = 0; k < min(sp, win); ++k) V.set_gstack(k, V.wstack(k));
        for (uint32_t k = 0; k < min(msize >> 2, mw); ++k) V.set_gmdw(k, V.lmdw(k));
        L.pc[lane] = pc; L.sp[lane] = sp; L.msize[lane] = msize; L.depth[lane] = depth;
        L.gas_min[lane] = gmin; L.gas_max[lane] = gmax;
        L.status[lane] = status; L.aux[lane] = aux;
        L.fent[lane] = fent;
        if (loop_on) L.trace_len[lane] = tlen;
        // HOOK_ACK covers one instruction: consumed once the lane has executed
        if (hook_ack && executed > 0u) L.flags[lane] = flags & ~LANE_HOOK_ACK;
        L.steps[lane] += executed;
        if (n_sha3) L.sha3_count[lane] += n_sha3;
        if (n_exp) L.exp_count[lane] += n_exp;
    }

#ifdef MG_K1_CLOCKS
    CLK_MARK(258u);
    if ((threadIdx.x & 63u) == 0u) {
        const uint32_t gw = blockIdx.x * (LANE_BLOCK / 64u) + (threadIdx.x >> 6);
        if (gw < 4096u)
            for (uint32_t i = 0; i < CLK_BINS; ++i) g_k1_clk[gw * CLK_BINS + i] = s_clk[threadIdx.x >> 6][i];
    }
#endif
#undef CLK_MARK
    if (staged && cov_on) {
        __syncthreads();
        const DevCode BC = codes[bcode];
        for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x)
            if (s_cov[i]) cov[BC.cov_off + i] = 1;
    }
    if (prof) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 260u; i += blockDim.x)
            if (s_prof[i]) atomicAdd(&prof[i], (unsigned long long)s_prof[i]);
    }
    // statistics: one plain store of the block's totals into ctr[blockIdx.x]
    // (the host sums the blocks).  Same-address atomics from every wave of the
    // grid serialise across the XCDs and cost ~20 us per launch at 1,024 waves.
    if (ctr) {
        __shared__ unsigned long long s_ctr[LANE_BLOCK / 64u][5];
        unsigned long long s = executed;
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
        const uint64_t b_run = __ballot(in_range && status == ST_RUNNING);
        const uint64_t b_hook = __ballot(in_range && status == ST_HOOK);
        const uint64_t b_esc = __ballot(in_range && status == ST_ESCAPE);
        const uint64_t b_all = __ballot(in_range);
        const uint32_t w = threadIdx.x >> 6;
        if ((threadIdx.x & 63u) == 0u) {
            s_ctr[w][0] = s;
            s_ctr[w][1] = __popcll(b_run);
            s_ctr[w][2] = __popcll(b_hook);
            s_ctr[w][3] = __popcll(b_esc);
            s_ctr[w][4] = __popcll(b_all);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long t[5] = {0, 0, 0, 0, 0};
            for (uint32_t k = 0; k < LANE_BLOCK / 64u; ++k)
                for (int j = 0; j < 5; ++j) t[j] += s_ctr[k][j];
            DevCounters c;
            c.lane_steps = t[0];
            c.running = (unsigned)t[1];
            c.hooked = (unsigned)t[2];
            c.escaped = (unsigned)t[3];
            c.halted = (unsigned)(t[4] - t[1] - t[2] - t[3]);
            ctr[blockIdx.x] = c;
        }
    }
}
