// bv_eval.cuh — kernel 2: constraint-set x candidate-model evaluation (prefilter).
//
// Replaces the model loop of ModelCache.check_quick_sat (support_utils.py:60-68):
// `for model in reversed(lru): if is_true(model.eval(And(constraints),
// model_completion=True)): return model`.  The host (mythril_amd/smt/flatten.py)
// compiles each constraint set into a straight-line register program over
// 256-bit values; this kernel evaluates every program against every model.
//
// Mapping: one thread = one candidate model; a workgroup stages a tile of
// programs in LDS and all its waves run the SAME instruction stream, so the op,
// operand kinds and widths are wave-uniform (readfirstlane -> scalar branches,
// no divergence); only the 256-bit values are per lane.  Results are reduced per
// wave with ballots: sat count (popc) and first satisfying model (ffs) per DAG.
//
// Instruction (4 x u32):
//   w0: op[0:8) | width[8:17) | store[17] | dst_slot[18:22)
//   w1, w2, w3: operand refs: kind[30:32) (0 acc, 1 slot, 2 var, 3 const) | index[0:30)
//               or immediates (EXTRACT lo, SEXT source width, CONCAT low width,
//               compare operand width), per op.
// The result always lands in the accumulator; `store` also writes slot dst.
// Only operand A may refer to the accumulator (the host flattener swaps or
// spills, bv_upload checks): A is then loaded INTO the accumulator's registers
// and the accumulator is dead for the rest of the instruction, so no operand
// copy of the 256-bit accumulator is needed per instruction.
#pragma once
#include <string>

#include "u256.cuh"
#include "../../include/mythgpu.h"

enum BvOp : uint32_t {
    BV_COPY = 0,       // acc = A
    BV_ADD, BV_SUB, BV_MUL, BV_UDIV, BV_UREM, BV_SDIV, BV_SREM, BV_SMOD,
    BV_AND, BV_OR, BV_XOR, BV_NOT, BV_NEG, BV_SHL, BV_LSHR, BV_ASHR,
    BV_EQ, BV_ULT, BV_ULE, BV_UGT, BV_UGE, BV_SLT, BV_SLE, BV_SGT, BV_SGE,   // w3 = operand width
    BV_BAND, BV_BOR, BV_BXOR, BV_BNOT, BV_BIMPLIES,
    BV_ITE,            // A cond, B then, C else
    BV_EXTRACT,        // A, w2 = lo
    BV_CONCAT,         // A high, B low, w3 = width of B
    BV_ZEXT,           // A (value already masked)
    BV_SEXT,           // A, w2 = source width
    BV_ADD_NOOVF_U,    // bvadd_noovfl unsigned; w3 = operand width
    BV_MUL_NOOVF_U,    // bvumul_noovfl;        w3 = operand width
    BV_SUB_NOUDF_U,    // BVSubNoUnderflow unsigned: b <= a
    BV_NE,             // w3 = operand width
    BV_TAB,            // A = key k0, B = key k1, w3 = table | part << 20 | lo << 21:
                       // bits [256 part + lo, +width) of the model's array / function
                       // interpretation at (k0, k1), else its default (lower.py)
    BV_UMIN, BV_UMAX,  // ite(cmp(A, B), A, B) folded by the compiler (flatten._fold_select)
    BV_SMIN, BV_SMAX,  // signed at `width`
    BV_RSUB,           // B - A           (operand-swapped forms: the accumulator is only
    BV_RCONCAT,        // A low, B high,   ever operand A; w3 = width of A)
    BV_NUM_OPS,
    // fused pairs, formed by bv_upload from adjacent instructions (never accepted
    // at the C-ABI): the first's result feeds only the second's accumulator, so one
    // dispatch does both and the 0/1 or 128-bit intermediate is never widened to
    // a 256-bit accumulator.  MG_BV_FUSE=0 uploads the programs unfused.
    BV_CMP_BAND = BV_NUM_OPS,   // cmp(A, B) & C: w0 bits 22..27 = the comparison, width = its
                                // operand width (w3 of the comparison); C = the and's B
    BV_EXT_RCAT,                // rconcat(extract(A, lo, ew), B): w3 = shift | lo << 9 | ew << 17
    BV_BIN2,                    // op2(op1(A, B), C) for two 256-bit ops of bv_simple: w0 bits
                                // 22..25 = op1, 26..29 = op2 (bv_simple indices); C = op2's B
    BV_BINX,                    // a chain of 3 or 4 such ops, two instruction slots: w0 bits
                                // 22..24 = the count, A, B1, B2; then {kinds 4 bits each, B3, B4, 0}
    BV_NUM_INTERNAL
};

#define BV_REF_ACC 0u
#define BV_REF_SLOT 1u
#define BV_REF_VAR 2u
#define BV_REF_CONST 3u
#define BV_MAX_SLOTS 16u    // 4-bit slot field; 16 slots = 128 KiB of LDS per block
#define BV_BLOCK 256u
#define BV_TILE_INSNS 2048u   // longest program (LDS tile upper bound: 32 KiB)
#ifndef BV_TILE_MIN
#define BV_TILE_MIN 256u      // smallest program tile (4 KiB in LDS)
#endif
#define BV_TILE_DAGS 64u      // most DAGs per tile (per-block result accumulators)
#define BV_GROUP_TARGET 4096u // blocks wanted per launch (16 per CU)

struct BvState {
    uint32_t n_dags = 0, n_models = 0, n_vars = 0, n_slots = 0, n_consts = 0, n_tiles = 0, tile_cap = 0;
    uint4 *insns = nullptr;          // [total]
    uint32_t *prog_off = nullptr;    // [n_dags + 1]
    uint32_t *tile_dag = nullptr;    // [n_tiles + 1] first DAG of each tile
    uint4 *consts = nullptr;         // [n_consts][2]
    uint4 *values = nullptr;         // [n_vars][n_models][2]
    uint32_t n_tables = 0, n_entries = 0;
    uint32_t *tab_start = nullptr;   // [n_tables][n_models]
    uint32_t *tab_count = nullptr;   // [n_tables][n_models]
    uint4 *tab_entries = nullptr;    // [n_entries][8]: k0, k1, value (512 bits)
    uint4 *tab_default = nullptr;    // [n_tables][n_models][4]
    uint32_t *first_sat = nullptr;   // [n_dags]
    uint32_t *sat_count = nullptr;   // [n_dags]
    unsigned long long *sat_bits = nullptr;   // [n_dags][bit_words] (mg_eval_bits)
    size_t cap_bits = 0;
    bool want_bits = false;
    size_t cap_insns = 0, cap_dags = 0, cap_consts = 0, cap_values = 0, cap_tiles = 0;
    size_t cap_entries = 0;
    std::vector<uint32_t> h_tiles;
    std::vector<uint32_t> h_insns, h_off;   // the fused programs (bv_fuse)
};

DEV U256 bv_mask(U256 v, uint32_t width) {
    if (width >= 256u) return v;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t lo = 32u * i;
        if (width <= lo) v.w[i] = 0u;
        else if (width < lo + 32u) v.w[i] &= (1u << (width - lo)) - 1u;
    }
    return v;
}
// sign-extend a width-bit value to 256 bits.  Per-limb selects on the (wave-
// uniform) width only: a runtime limb index would put the value in scratch.
DEV U256 bv_sext(U256 v, uint32_t width) {
    if (width >= 256u || width == 0u) return v;
    const uint32_t sb = width - 1u, li = sb >> 5, bi = sb & 31u;
    uint32_t top = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) top |= ((uint32_t)i == li) ? v.w[i] : 0u;
    if (!((top >> bi) & 1u)) return v;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t lo = 32u * i;
        if (width <= lo) v.w[i] = 0xffffffffu;
        else if (width < lo + 32u) v.w[i] |= 0xffffffffu << (width - lo);
    }
    return v;
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

struct BvTables {
    const uint32_t *__restrict__ start;
    const uint32_t *__restrict__ count;
    const uint4 *__restrict__ entries;
    const uint4 *__restrict__ dflt;
};

// Per lane, the context is two VGPRs: m = chunk * BV_BLOCK + tid (the model
// this thread evaluates, unclamped) and the LDS address of the thread's slot
// column (tid = m % BV_BLOCK, the same for every chunk: a slot access adds only
// the slot's uniform offset, one VALU).  The value / table rows use
// min(m, n_models - 1) (a dead lane past the pool reads the last model; its
// result is masked).  Keeping model, tid and the live flag as separate VGPRs
// spilled them at 64 VGPRs inside the DAG loop in round 2 (12.6 GB of scratch
// traffic per C4 launch, profiles/r02/traffic.json); this build fits in 61.
struct BvCtx {
    const uint4 *__restrict__ values;
    const uint4 *__restrict__ consts;
    uint4 *lane_slots;     // LDS [n_slots][2][BV_BLOCK], at this thread's column (+ tid)
    uint32_t n_models, m;
    BvTables tab;
    DEV uint32_t model() const { return min(m, n_models - 1u); }
};

DEV U256 ld2(const uint4 *p) {
    const uint4 x = p[0], y = p[1];
    U256 r;
    r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
    r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
    return r;
}

// Equality and zero tests as one VALU reduction and one compare.  Written plainly
// (u256.cuh), instcombine turns (x0 | .. | x7) == 0 into eight per-limb compares
// whose lane masks are joined by seven scalar s_or_b64 / s_and_b64 -- scalar issue,
// which this kernel is bound by; the empty asm keeps the reduction in a VGPR.
DEV bool bv_zero32(uint32_t o) {
    asm volatile("" : "+v"(o));
    return o == 0u;
}
DEV bool bv_eq(const U256 &a, const U256 &b) {
    uint32_t o = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.w[i] ^ b.w[i];
    return bv_zero32(o);
}
DEV bool bv_iszero(const U256 &a) {
    uint32_t o = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.w[i];
    return bv_zero32(o);
}
DEV bool bv_fits32(const U256 &a) {
    uint32_t o = 0u;
#pragma unroll
    for (int i = 1; i < 8; ++i) o |= a.w[i];
    return bv_zero32(o);
}

// model interpretation lookup (entries are unique keys: first match wins)
DEV U256 bv_table(const BvCtx &c, const U256 &k0, const U256 &k1, uint32_t imm) {
    const uint32_t t = imm & 0xfffffu, part = (imm >> 20) & 1u, lo = (imm >> 21) & 0xffu;
    const size_t tm = (size_t)t * c.n_models + c.model();
    const uint32_t s0 = c.tab.start[tm], cnt = c.tab.count[tm];
    U256 v = ld2(c.tab.dflt + tm * 4u + part * 2u);
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint4 *e = c.tab.entries + (size_t)(s0 + k) * 8u;
        if (bv_eq(ld2(e), k0) && bv_eq(ld2(e + 2), k1)) {
            v = ld2(e + 4 + part * 2u);
            break;
        }
    }
    return lo ? u_shr_u(v, lo, 0u) : v;      // lo: uniform immediate
}

// An operand's 256 bits from a slot (LDS), a variable (the model's value row)
// or a constant (uniform address: scalar loads).  Each path ends in its own
// opaque asm: the three paths' loads are then no longer identical trailing
// instructions, so the compiler cannot sink them into one generic-pointer
// load after the branch (it did, as eight per-dword flat_loads, once A's fetch
// wrote the accumulator's registers).  The accumulator itself is never
// fetched here (operand A = the accumulator is handled by the caller).
#define BV_PIN(tag_, r_) asm volatile(tag_ : "+v"((r_).w[0]), "+v"((r_).w[1]), "+v"((r_).w[2]), "+v"((r_).w[3]), \
                                      "+v"((r_).w[4]), "+v"((r_).w[5]), "+v"((r_).w[6]), "+v"((r_).w[7]))
DEV U256 bv_fetch(const BvCtx &c, uint32_t ref) {
    const uint32_t kind = ref >> 30, idx = ref & 0x3fffffffu;
    U256 r;
    if (kind == BV_REF_VAR) {            // the commonest B operand (C4: 46 %) first
        // a 32-bit byte offset from the table's base (bv_upload keeps the table
        // under 4 GiB): the uniform part is one scalar multiply, the load takes the
        // base as its SGPR address
        const uint32_t off = (idx * c.n_models + c.model()) * 32u;
        const uint4 *p = reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(c.values) + off);
        const uint4 x = p[0], y = p[1];
        r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
        r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
        BV_PIN("; variable operand", r);
        return r;
    }
    if (kind <= BV_REF_SLOT) {
        const uint4 x = c.lane_slots[(idx * 2u) * BV_BLOCK];
        const uint4 y = c.lane_slots[(idx * 2u + 1u) * BV_BLOCK];
        r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
        r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
        BV_PIN("; slot operand", r);
        return r;
    }
    // constant: uniform address -> scalar loads, at a 32-bit byte offset the load
    // takes in an SGPR (bv_upload: the constant table is far below 4 GiB)
    const uint4 *p = reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(c.consts) + (idx << 5));
    const uint4 x = p[0], y = p[1];
    r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
    r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
    BV_PIN("; constant operand", r);
    return r;
}

// The division-class ops go through TWO inlined u_divmod_nz sites instead of
// six: UDIV/UREM (bv_udivrem), and SDIV SREM SMOD MUL_NOOVF_U (bv_divop:
// operands prepared per op -- sign-extend + magnitude for the signed ops,
// (2^w-1, A) for the overflow test -- divided once, the quotient / remainder
// post-processed per op).  Six inlined copies of Knuth D doubled the kernel's
// code; one shared site kept the divisor live across the division and spilled
// inside it (divrem class 83 -> 92 ms, profiles/r03/k2).  z3 semantics for a zero divisor are kept:
// udiv -> ones, urem/srem/smod -> a, sdiv -> (a < 0 ? 1 : -1).
// UDIV/UREM (C4's division class) keep nothing live across the division; the
// signed ops and the overflow test share the second site
DEV U256 bv_udivrem(bool quotient, const U256 &A, const U256 &B) {
    U256 q = u_ones(), r = A;                   // b == 0: bvudiv -> ones, bvurem -> a
    if (!bv_iszero(B)) u_divmod_nz_t<true>(A, B, q, r);
    return quotient ? q : r;
}
#define BV_DIV_OPS ((1ull << BV_SDIV) | (1ull << BV_SREM) | (1ull << BV_SMOD) | (1ull << BV_MUL_NOOVF_U))
DEV U256 bv_divop(uint32_t op, uint32_t width, uint32_t rc, const U256 &A, const U256 &B) {
    const bool sgn = op == BV_SDIV || op == BV_SREM || op == BV_SMOD;   // wave-uniform
    U256 a = A, b = B;
    bool na = false, nb = false;
    if (sgn) {                                  // magnitudes of the width-bit signed operands
        a = bv_sext(A, width);
        b = bv_sext(B, width);
        na = u_isneg(a);
        nb = u_isneg(b);
        if (na) a = u_neg(a);
        if (nb) b = u_neg(b);
    }
    U256 keep = b;                              // divisor magnitude (SMOD) / B (MUL_NOOVF_U)
    if (op == BV_MUL_NOOVF_U) { keep = B; b = A; a = bv_mask(u_ones(), rc); }
    const bool bz = bv_iszero(b);
    U256 q = u_ones(), r = a;                   // b == 0: q = ones, r = a
    if (!bz) u_divmod_nz_t<true>(a, b, q, r);
    switch (op) {
    case BV_UDIV: return q;
    case BV_UREM: return r;
    case BV_SDIV: return bz ? (na ? u_small(1) : u_ones()) : ((na != nb) ? u_neg(q) : q);
    case BV_SREM: return na ? u_neg(r) : r;     // b == 0: the signed dividend
    case BV_SMOD: {
        const U256 s = na ? u_neg(r) : r;       // srem: sign of the dividend
        if (bz || bv_iszero(s) || u_isneg(s) == nb) return s;
        return u_add(s, nb ? u_neg(keep) : keep);   // smod: sign of the divisor
    }
    default:                                    // MUL_NOOVF_U: a*b <= 2^w-1 <=> b <= floor((2^w-1)/a)
        return u_small(!u_lt(q, keep));         // a == 0: q = ones; b == 0: never less
    }
}

// ops whose 256-bit result may have bits at or above `width`: only these are
// masked (the comparisons, Boolean connectives and overflow tests produce 0/1)
#define BV_MASK_OPS ((1ull << BV_COPY) | (1ull << BV_ADD) | (1ull << BV_SUB) | (1ull << BV_MUL) | \
                     (1ull << BV_UDIV) | (1ull << BV_SDIV) | (1ull << BV_SREM) | (1ull << BV_SMOD) | \
                     (1ull << BV_NOT) | (1ull << BV_NEG) | (1ull << BV_SHL) | (1ull << BV_ASHR) | \
                     (1ull << BV_EXTRACT) | (1ull << BV_CONCAT) | (1ull << BV_SEXT) | (1ull << BV_ITE) | \
                     (1ull << BV_TAB) | (1ull << BV_SMIN) | (1ull << BV_SMAX) | (1ull << BV_ZEXT) | \
                     (1ull << BV_AND) | (1ull << BV_OR) | (1ull << BV_XOR) | (1ull << BV_LSHR) | \
                     (1ull << BV_UREM) | (1ull << BV_UMIN) | (1ull << BV_UMAX) | (1ull << BV_RSUB) | \
                     (1ull << BV_RCONCAT) | (1ull << BV_EXT_RCAT))

// Predecode (bv_predecode, at upload, after bv_fuse): flags the kernel tests
// with one scalar bit test instead of deriving them from op and width per
// instruction -- op byte bit 7: the op has one operand (no B fetch, the small
// switch); w0 bit 30: the result is masked to `width` (width < 256 and the op
// in BV_MASK_OPS).  Internal to the library: the C-ABI's programs never carry
// them (bv_upload rejects bits 22..31, and op < BV_NUM_OPS < 128).
#define BV_W0_UNARY 0x80u
#define BV_W0_HOT 0x40u
#define BV_W0_MASK (1u << 30)
static bool bv_is_unary(uint32_t op) {
    return op == BV_COPY || op == BV_NOT || op == BV_NEG || op == BV_BNOT || op == BV_EXTRACT || op == BV_ZEXT ||
           op == BV_SEXT;
}
static void bv_predecode(std::vector<uint32_t> &v, const std::vector<uint32_t> &off, uint32_t n) {
    for (uint32_t d = 0; d < n; ++d) {
        for (uint32_t i = off[d]; i < off[d + 1]; ++i) {
            uint32_t &w0 = v[4 * (size_t)i];
            const uint32_t op = w0 & 0xffu, width = (w0 >> 8) & 0x1ffu;
            if (bv_is_unary(op)) w0 |= BV_W0_UNARY;
            // each group's commonest op (C4: extract 13 % of the fused instructions,
            // cmp-and 19 %) is tested by this bit before the group's switch
            if (op == BV_EXTRACT || op == BV_CMP_BAND) w0 |= BV_W0_HOT;
            if (width < 256u && op < 64u && ((BV_MASK_OPS >> op) & 1ull)) w0 |= BV_W0_MASK;
            if (op == BV_BINX || (w0 >> 31)) ++i;      // skip the extension slot
        }
    }
}

// MG_BV_WAVES: minimum waves per SIMD the register allocation must allow (0
// leaves the compiler's choice).  8 caps the kernel at 64 VGPRs (a few spill to
// scratch); with the scalar-load instruction fetch the block's LDS is its 16 KiB of
// slots, so 8 blocks fit a CU: C4 249 -> 220 ms (profiles/r02/ab_k2_occupancy.log)
#ifndef MG_BV_WAVES
#define MG_BV_WAVES 8
#endif
#if MG_BV_WAVES
#define BV_BOUNDS __launch_bounds__(BV_BLOCK, MG_BV_WAVES)
#else
#define BV_BOUNDS __launch_bounds__(BV_BLOCK)
#endif

// the 256-bit binary ops BV_BIN2 fuses (index = position in kBvSimple), each
// exactly as the unfused switch computes it
__device__ __forceinline__ U256 bv_simple(uint32_t k, const U256 &a, const U256 &b) {
    switch (k) {                                   // wave-uniform
    case 0: return u_add(a, b);
    case 1: return u_sub(a, b);
    case 2: return u_mul(a, b);
    case 3: return u_and(a, b);
    case 4: return u_or(a, b);
    case 5: return u_xor(a, b);
    case 6: return u_select(u_lt(a, b), b, a);     // BV_UMAX
    case 7: return u_select(u_lt(b, a), b, a);     // BV_UMIN
    default: return u_sub(b, a);                   // BV_RSUB
    }
}
static const uint32_t kBvSimple[9] = {BV_ADD, BV_SUB, BV_MUL, BV_AND, BV_OR, BV_XOR, BV_UMAX, BV_UMIN, BV_RSUB};

__global__ BV_BOUNDS void k_bv_eval(const uint4 *__restrict__ insns,
                                                      const uint32_t *__restrict__ prog_off,
                                                      const uint32_t *__restrict__ tile_dag,
                                                      const uint4 *__restrict__ consts,
                                                      const uint4 *__restrict__ values, uint32_t n_models,
                                                      BvTables tab,
                                                      uint32_t n_slots, uint32_t tile_first, uint32_t n_tiles,
                                                      uint32_t tiles_pad, uint32_t dag_lo, uint32_t dag_hi,
                                                      uint32_t tile_cap, uint32_t chunks_per_block,
                                                      uint32_t *__restrict__ first_sat,
                                                      uint32_t *__restrict__ sat_count,
                                                      unsigned long long *__restrict__ sat_bits,
                                                      uint32_t bit_words) {
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    // instructions are read with scalar loads (uniform address -> s_load_dwordx4
    // through the scalar cache); LDS holds only the register slots.  Staging the
    // program tile in LDS measured slower (occupancy, ab/k2_lds_fetch.diff)
    uint4 *slots = smem;                         // [n_slots][2][BV_BLOCK]
    // group-major order with the tile count padded to a multiple of 8: the blocks
    // of one program tile share blockIdx % 8, i.e. one XCD's L2 (speed only)
    const uint32_t b = blockIdx.x;
    const uint32_t tile = tile_first + (b % tiles_pad);
    const uint32_t group = b / tiles_pad;
    if (tile >= tile_first + n_tiles) return;
    const uint32_t d0 = max(tile_dag[tile], dag_lo), d1 = min(tile_dag[tile + 1], dag_hi);
    if (d0 >= d1) return;
    // the tile is read from HBM once per block and reused for every model chunk
    const uint32_t i0 = prog_off[d0], i1 = prog_off[d1];
    // per-block results of the tile's DAGs: waves combine in LDS, the block adds
    // its totals to HBM once per DAG (not one atomic pair per wave per DAG)
    __shared__ uint32_t blk_cnt[BV_TILE_DAGS], blk_first[BV_TILE_DAGS];
    if (threadIdx.x < BV_TILE_DAGS) { blk_cnt[threadIdx.x] = 0u; blk_first[threadIdx.x] = 0xffffffffu; }
    __syncthreads();

    const uint32_t n_chunks = (n_models + BV_BLOCK - 1u) / BV_BLOCK;
    const uint32_t c_lo = group * chunks_per_block, c_hi = min(c_lo + chunks_per_block, n_chunks);
    // thread index = the wave's first (an SGPR) + the lane id (v_mbcnt): nothing
    // keeps threadIdx.x alive across the loops
    const uint32_t wave0 = uni(threadIdx.x) & ~63u;
    // this thread's column of the slot table (tid = m % BV_BLOCK = wave0 + lane for every
    // chunk): a slot access adds only the slot's uniform offset
    uint4 *const lane_slots = slots + wave0 + __lane_id();
    // DAG-major: one DAG's program (tens of instructions) is evaluated for all of
    // the block's model chunks while it is hot in the scalar cache; chunk-major
    // re-read the whole tile (up to 32 KiB) once per chunk, which the scalar
    // cache cannot hold and a CU's resident blocks' tiles overflow L2 with
    for (uint32_t d = d0; d < d1; ++d) {
    const uint32_t p0 = prog_off[d] - i0, p1 = prog_off[d + 1] - i0;
    for (uint32_t chunk = c_lo; chunk < c_hi; ++chunk) {
        BvCtx c{values, consts, lane_slots, n_models, chunk * BV_BLOCK + wave0 + __lane_id(), tab};
        U256 acc = u_zero();
        // byte offsets into the tile (32-bit, wave-uniform): the scalar load takes the
        // offset as its SGPR operand instead of a 64-bit address computed per instruction
        const char *const tileb = reinterpret_cast<const char *>(insns + i0);
        for (uint32_t off = p0 << 4, off_end = p1 << 4; off < off_end; off += 16u) {
            // c.m is the only per-lane context.  Round 3 hid its loop invariance
            // (an empty asm on it here) because min(m, n - 1) and m % 256 kept in
            // VGPRs across the loop spilled; with the predecoded dispatch the
            // kernel fits without it (62 VGPRs, no scratch) and runs 1.9 % faster
            // with them hoisted (profiles/r05/k2/ab_k2_q.log)
            uint32_t w0, ra, rb, rc;
            {
                const uint4 ins = *reinterpret_cast<const uint4 *>(tileb + uni(off));
                w0 = ins.x; ra = ins.y; rb = ins.z; rc = ins.w;
            }
            // op byte bit 7 = one operand (bv_predecode); w0 bit 30 = mask to width
            const uint32_t op = w0 & 0x3fu, width = (w0 >> 8) & 0x1ffu;
            if ((ra >> 30) != BV_REF_ACC) acc = bv_fetch(c, ra);    // A in the accumulator's registers
            const U256 A = acc;
            U256 r;
            if (w0 & BV_W0_UNARY) {
                if (w0 & BV_W0_HOT) {
                    r = u_shr_u(A, rb & 0xffu, 0u);                              // BV_EXTRACT
                } else {
                switch (op) {
                case BV_NOT: r = u_not(A); break;
                case BV_NEG: r = u_neg(A); break;
                case BV_BNOT: r = u_small((A.w[0] & 1u) ^ 1u); break;
                case BV_SEXT: r = bv_sext(A, rb); break;
                default: r = A; break;                                          // BV_COPY, BV_ZEXT
                }
                }
            } else {
                U256 B = bv_fetch(c, rb);
                if (w0 & BV_W0_HOT) {                        // BV_CMP_BAND
                    const uint32_t sub = (w0 >> 22) & 0x3fu;
                    bool t;
                    switch (sub) {
                    case BV_EQ: t = bv_eq(A, B); break;
                    case BV_NE: t = !bv_eq(A, B); break;
                    case BV_ULT: t = u_lt(A, B); break;
                    case BV_ULE: t = !u_lt(B, A); break;
                    case BV_UGT: t = u_lt(B, A); break;
                    case BV_UGE: t = !u_lt(A, B); break;
                    case BV_SLT: t = u_slt(bv_sext(A, width), bv_sext(B, width)); break;
                    case BV_SLE: t = !u_slt(bv_sext(B, width), bv_sext(A, width)); break;
                    case BV_SGT: t = u_slt(bv_sext(B, width), bv_sext(A, width)); break;
                    default: t = !u_slt(bv_sext(A, width), bv_sext(B, width)); break;   // BV_SGE
                    }
                    const U256 C = bv_fetch(c, rc);
                    r = u_small((t ? 1u : 0u) & C.w[0]);
                } else if (op == BV_UDIV || op == BV_UREM) {        // the unsigned division site
                    r = bv_udivrem(op == BV_UDIV, A, B);
                } else if ((BV_DIV_OPS >> op) & 1ull) {      // the signed / overflow site
                    r = bv_divop(op, width, rc, A, B);
                } else {
                switch (op) {
                case BV_ADD: r = u_add(A, B); break;
                case BV_SUB: r = u_sub(A, B); break;
                case BV_MUL: r = u_mul(A, B); break;
                case BV_AND: r = u_and(A, B); break;
                case BV_OR: r = u_or(A, B); break;
                case BV_XOR: r = u_xor(A, B); break;
                case BV_SHL: case BV_LSHR: case BV_ASHR: {
                    // a constant shift amount is wave-uniform: scalar-branch shifts
                    const bool ub = (rb >> 30) == BV_REF_CONST;
                    const bool in = bv_fits32(B) && B.w[0] < width;
                    if (op == BV_ASHR) {
                        const U256 sa = bv_sext(A, width);
                        const uint32_t fill = u_isneg(sa) ? 0xffffffffu : 0u;
                        if (ub) {
                            const uint32_t sh = uni(in ? B.w[0] : 255u);
                            r = u_shr_u(sa, sh, fill);
                        } else {
                            r = u_shr_n(sa, in ? B.w[0] : 255u, fill);
                        }
                    } else if (ub) {
                        if (!uni(in ? 1u : 0u)) r = u_zero();
                        else if (op == BV_SHL) r = u_shl_u(A, uni(B.w[0]));
                        else r = u_shr_u(A, uni(B.w[0]), 0u);
                    } else {
                        r = !in ? u_zero() : op == BV_SHL ? u_shl_n(A, B.w[0]) : u_shr_n(A, B.w[0], 0u);
                    }
                    break;
                }
                case BV_EQ: r = u_small(bv_eq(A, B)); break;
                case BV_NE: r = u_small(!bv_eq(A, B)); break;
                case BV_ULT: r = u_small(u_lt(A, B)); break;
                case BV_ULE: r = u_small(!u_lt(B, A)); break;
                case BV_UGT: r = u_small(u_lt(B, A)); break;
                case BV_UGE: r = u_small(!u_lt(A, B)); break;
                case BV_SLT: r = u_small(u_slt(bv_sext(A, rc), bv_sext(B, rc))); break;
                case BV_SLE: r = u_small(!u_slt(bv_sext(B, rc), bv_sext(A, rc))); break;
                case BV_SGT: r = u_small(u_slt(bv_sext(B, rc), bv_sext(A, rc))); break;
                case BV_SGE: r = u_small(!u_slt(bv_sext(A, rc), bv_sext(B, rc))); break;
                case BV_BAND: r = u_small(A.w[0] & B.w[0] & 1u); break;
                case BV_BOR: r = u_small((A.w[0] | B.w[0]) & 1u); break;
                case BV_BXOR: r = u_small((A.w[0] ^ B.w[0]) & 1u); break;
                case BV_BIMPLIES: r = u_small(((A.w[0] & 1u) ^ 1u) | (B.w[0] & 1u)); break;
                case BV_ITE: {
                    const U256 C = bv_fetch(c, rc);
                    r = u_select((A.w[0] & 1u) != 0u, B, C);
                    break;
                }
                case BV_CONCAT: r = u_or(u_shl_u(A, rc), B); break;                 // rc: uniform
                case BV_ADD_NOOVF_U: {  // top bit of the (w+1)-bit sum is 0
                    const U256 s = u_add(A, B);
                    const bool ovf = rc >= 256u ? u_lt(s, A) : !bv_iszero(u_shr_u(s, rc, 0u));
                    r = u_small(!ovf);
                    break;
                }
                case BV_SUB_NOUDF_U: r = u_small(!u_lt(A, B)); break;
                case BV_TAB: r = bv_table(c, A, B, rc); break;
                case BV_UMIN: r = u_select(u_lt(B, A), B, A); break;
                case BV_UMAX: r = u_select(u_lt(A, B), B, A); break;
                case BV_SMIN: r = u_select(u_slt(bv_sext(B, width), bv_sext(A, width)), B, A); break;
                case BV_SMAX: r = u_select(u_slt(bv_sext(A, width), bv_sext(B, width)), B, A); break;
                case BV_RSUB: r = u_sub(B, A); break;
                case BV_RCONCAT: r = u_or(u_shl_u(B, rc), A); break;
                case BV_BIN2: {
                    const U256 t = bv_simple((w0 >> 22) & 0xfu, A, B);
                    const U256 C = bv_fetch(c, rc);
                    r = bv_simple((w0 >> 26) & 0xfu, t, C);
                    break;
                }
                case BV_BINX: {
                    uint32_t e0, e1, e2;
                    {
                        const uint4 x = *reinterpret_cast<const uint4 *>(tileb + uni(off + 16u));
                        e0 = x.x; e1 = x.y; e2 = x.z;
                    }
                    off += 16u;                              // the extension slot
                    const uint32_t k = (w0 >> 22) & 0x7u;
                    U256 t = bv_simple(e0 & 0xfu, A, B);
#pragma unroll 1
                    for (uint32_t j = 1; j < k; ++j) {
                        const uint32_t ref = j == 1u ? rc : j == 2u ? e1 : e2;
                        const U256 C = bv_fetch(c, ref);
                        t = bv_simple((e0 >> (4u * j)) & 0xfu, t, C);
                    }
                    r = t;
                    break;
                }
                case BV_EXT_RCAT: {
                    const uint32_t ew = (rc >> 17) & 0x1ffu;
                    U256 lo = u_shr_u(A, (rc >> 9) & 0xffu, 0u);
                    if (ew < 256u) lo = bv_mask(lo, ew);
                    r = u_or(u_shl_u(B, rc & 0x1ffu), lo);
                    break;
                }
                default: r = u_zero(); break;
                }
            }
            }
            // mask, fused tail and store in one test for the common instruction
            // that has none of them
            if (w0 & (BV_W0_MASK | (1u << 31) | (1u << 17))) {
                // the result masked to its width first (a tail's ops are 256-bit)
                if (w0 & BV_W0_MASK) r = bv_mask(r, width);
                if (w0 >> 31) {
                    // fused tail (bv_fuse): 1-3 bv_simple ops applied to this result,
                    // from an extension slot {kinds | count << 28, B1, B2, B3}
                    uint32_t e0, e1, e2, e3;
                    {
                        const uint4 x = *reinterpret_cast<const uint4 *>(tileb + uni(off + 16u));
                        e0 = x.x; e1 = x.y; e2 = x.z; e3 = x.w;
                    }
                    off += 16u;
                    const uint32_t k = e0 >> 28;
#pragma unroll 1
                    for (uint32_t j = 0; j < k; ++j) {
                        const uint32_t ref = j == 0u ? e1 : j == 1u ? e2 : e3;
                        const U256 C = bv_fetch(c, ref);
                        r = bv_simple((e0 >> (4u * j)) & 0xfu, r, C);
                    }
                }
                if ((w0 >> 17) & 1u) {
                    const uint32_t ds = (w0 >> 18) & 0xfu;
                    lane_slots[(ds * 2u) * BV_BLOCK] = make_uint4(r.w[0], r.w[1], r.w[2], r.w[3]);
                    lane_slots[(ds * 2u + 1u) * BV_BLOCK] = make_uint4(r.w[4], r.w[5], r.w[6], r.w[7]);
                }
            }
            acc = r;
        }
        const bool sat = c.m < n_models && (acc.w[0] & 1u);
        const uint64_t bal = __ballot(sat);
        // the wave's first model, wave-uniform (an SGPR: nothing per lane stays live
        // across the DAG loop but c.m and the accumulator)
        const uint32_t wm = uni(c.m) & ~63u;
        if (bal && __lane_id() == 0u) {
            // optional per-model bitmap (one u64 per wave): lets the host replay
            // sequential check_quick_sat calls whose LRU bumps reorder the pool
            if (sat_bits) sat_bits[(size_t)d * bit_words + (wm >> 6)] = bal;
            atomicAdd(&blk_cnt[d - d0], (uint32_t)__popcll(bal));
            atomicMin(&blk_first[d - d0], wm + (uint32_t)(__ffsll((long long)bal) - 1));
        }
    }
    }
    __syncthreads();
    const uint32_t tid = wave0 + __lane_id();
    if (tid < d1 - d0) {
        const uint32_t n = blk_cnt[tid], f = blk_first[tid];
        if (n) {
            atomicAdd(&sat_count[d0 + tid], n);
            atomicMin(&first_sat[d0 + tid], f);
        }
    }
}


template <class T>
static int bv_ensure(T *&p, size_t &cap, size_t need) {
    if (need <= cap && p) return 0;
    hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, std::max<size_t>(need, 1) * sizeof(T)) != hipSuccess) return MG_ENOMEM;
    cap = std::max<size_t>(need, 1);
    return 0;
}

static void bv_free(BvState &s) {
    hipFree(s.insns); hipFree(s.prog_off); hipFree(s.tile_dag); hipFree(s.consts);
    hipFree(s.values); hipFree(s.first_sat); hipFree(s.sat_count);
    hipFree(s.tab_start); hipFree(s.tab_count); hipFree(s.tab_entries); hipFree(s.tab_default);
    hipFree(s.sat_bits);
    s = BvState{};
}

// Superinstructions: rewrite each DAG's program, fusing an instruction whose
// result is not stored into the next one when that one reads it as its
// accumulator and the pair is one of the flattener's common shapes (of C4's
// instructions, 10 % are a comparison feeding a Boolean and, 17 % a 256-bit
// add/sub/mul/and/or/xor/umax/umin/rsub feeding another (chains of 3 or 4 in one
// two-slot BV_BINX), 3 % a 128-bit extract feeding an rconcat; any other 256-bit
// op feeding 1-3 such binary ops takes them as a tail in an extension slot).  The fused program computes the same value bit for bit
// (tests/test_gpu_eval.py checks every program against the oracle, which runs
// the unfused program); it only saves a dispatch and the widening of the
// intermediate to a 256-bit accumulator.
static int bv_simple_index(uint32_t op) {
    for (int k = 0; k < 9; ++k)
        if (kBvSimple[k] == op) return k;
    return -1;
}
static void bv_fuse(const mg_dag_batch *dags, std::vector<uint32_t> &out, std::vector<uint32_t> &off,
                    bool bin2, bool binx, bool tail, bool narrow_tail) {
    const uint32_t n = dags->n_dags;
    out.clear();
    out.reserve((size_t)dags->prog_off[n] * 4);
    off.assign((size_t)n + 1, 0u);
    for (uint32_t d = 0; d < n; ++d) {
        off[d] = (uint32_t)(out.size() / 4);
        const uint32_t a = dags->prog_off[d], b = dags->prog_off[d + 1];
        for (uint32_t i = a; i < b; ++i) {
            const uint32_t *p = dags->insns + 4 * (size_t)i;
            const uint32_t op = p[0] & 0xffu;
            if (i + 1 < b && ((p[0] >> 17) & 1u) == 0u) {
                const uint32_t *q = p + 4;
                const uint32_t op2 = q[0] & 0xffu, w2 = (q[0] >> 8) & 0x1ffu;
                const uint32_t keep2 = q[0] & (0x1fu << 17);          // the second's store bit + slot
                const bool acc2 = (q[1] >> 30) == BV_REF_ACC;
                const bool cmp = (op >= BV_EQ && op <= BV_SGE) || op == BV_NE;
                if (acc2 && cmp && op2 == BV_BAND && p[3] >= 1u && p[3] <= 256u) {
                    const uint32_t w = (p[3] & 0x1ffu);
                    const uint32_t f[4] = {BV_CMP_BAND | (w << 8) | keep2 | (op << 22), p[1], p[2], q[2]};
                    out.insert(out.end(), f, f + 4);
                    ++i;
                    continue;
                }
                const int s1 = bv_simple_index(op), s2 = bv_simple_index(op2);
                const uint32_t w1 = (p[0] >> 8) & 0x1ffu;
                if (acc2 && s1 >= 0 && s2 >= 0 && w1 == 256u && w2 == 256u && bin2) {
                    // the longest chain (up to 4) of such ops, each feeding the next's
                    // accumulator unstored
                    uint32_t L = 2, kinds = (uint32_t)s1 | ((uint32_t)s2 << 4);
                    while (binx && L < 4 && i + L < b && ((dags->insns[4 * (size_t)(i + L - 1)] >> 17) & 1u) == 0u) {
                        const uint32_t *x = dags->insns + 4 * (size_t)(i + L);
                        const int sx = bv_simple_index(x[0] & 0xffu);
                        if (sx < 0 || ((x[0] >> 8) & 0x1ffu) != 256u || (x[1] >> 30) != BV_REF_ACC) break;
                        kinds |= (uint32_t)sx << (4 * L);
                        ++L;
                    }
                    if (L > 2) {
                        const uint32_t *last = dags->insns + 4 * (size_t)(i + L - 1);
                        const uint32_t f[8] = {BV_BINX | (256u << 8) | (last[0] & (0x1fu << 17)) | (L << 22),
                                               p[1], p[2], q[2],
                                               kinds, p[10], L > 3 ? p[14] : 0u, 0u};
                        out.insert(out.end(), f, f + 8);
                        i += L - 1;
                        continue;
                    }
                    const uint32_t f[4] = {BV_BIN2 | (256u << 8) | keep2 | ((uint32_t)s1 << 22) | ((uint32_t)s2 << 26),
                                           p[1], p[2], q[2]};
                    out.insert(out.end(), f, f + 4);
                    ++i;
                    continue;
                }
                if (acc2 && tail && (s1 < 0 || w1 != 256u) && (w1 == 256u || narrow_tail) && op < BV_NUM_OPS &&
                    s2 >= 0 && w2 == 256u) {
                    // any other op whose result feeds 1-3 256-bit bv_simple ops: the
                    // op keeps its own encoding, w0 bit 31 marks an extension slot
                    uint32_t L = 1, kinds = (uint32_t)s2;
                    while (L < 3 && i + L + 1 < b && ((dags->insns[4 * (size_t)(i + L)] >> 17) & 1u) == 0u) {
                        const uint32_t *x = dags->insns + 4 * (size_t)(i + L + 1);
                        const int sx = bv_simple_index(x[0] & 0xffu);
                        if (sx < 0 || ((x[0] >> 8) & 0x1ffu) != 256u || (x[1] >> 30) != BV_REF_ACC) break;
                        kinds |= (uint32_t)sx << (4 * L);
                        ++L;
                    }
                    const uint32_t *last = dags->insns + 4 * (size_t)(i + L);
                    const uint32_t f[8] = {(p[0] & ~(0x1fu << 17)) | (last[0] & (0x1fu << 17)) | (1u << 31),
                                           p[1], p[2], p[3],
                                           kinds | (L << 28), q[2], L > 1 ? p[10] : 0u, L > 2 ? p[14] : 0u};
                    out.insert(out.end(), f, f + 8);
                    i += L;
                    continue;
                }
                if (acc2 && op == BV_EXTRACT && op2 == BV_RCONCAT && q[3] < 512u) {
                    const uint32_t ew = (p[0] >> 8) & 0x1ffu;
                    const uint32_t f[4] = {BV_EXT_RCAT | (w2 << 8) | keep2, p[1], q[2],
                                           q[3] | ((p[2] & 0xffu) << 9) | (ew << 17)};
                    out.insert(out.end(), f, f + 4);
                    ++i;
                    continue;
                }
            }
            out.insert(out.end(), p, p + 4);
        }
    }
    off[n] = (uint32_t)(out.size() / 4);
}

static int bv_upload(BvState &s, const mg_dag_batch *dags, const mg_model_batch *models, hipStream_t st,
                     std::string &msg) {
    if (dags->n_dags == 0 || !dags->prog_off || !dags->insns) { msg = "empty DAG batch"; return MG_EINVAL; }
    if (dags->n_slots > BV_MAX_SLOTS) { msg = "too many slots"; return MG_EINVAL; }
    if ((uint64_t)dags->n_consts * 32u >= (1ull << 32)) { msg = "constant table over 4 GiB"; return MG_EINVAL; }
    if (models->n_models == 0 || (models->n_vars && !models->values)) { msg = "empty model batch"; return MG_EINVAL; }
    if ((uint64_t)models->n_vars * models->n_models * 32u >= (1ull << 32)) {
        msg = "model values over 4 GiB (variables x models x 32 bytes)";     // the kernel's 32-bit offsets
        return MG_EINVAL;
    }
    const uint32_t n = dags->n_dags;
    const uint32_t total = dags->prog_off[n];
    // validate programs on the host: refs in range, program fits a tile
    for (uint32_t d = 0; d < n; ++d) {
        const uint32_t a = dags->prog_off[d], b = dags->prog_off[d + 1];
        if (b < a || b - a > BV_TILE_INSNS || b > total) { msg = "bad program offsets / program too long"; return MG_EINVAL; }
    }
    for (uint32_t i = 0; i < total; ++i) {
        const uint32_t *w = dags->insns + 4 * (size_t)i;
        const uint32_t op = w[0] & 0xffu, width = (w[0] >> 8) & 0x1ffu;
        if (op >= BV_NUM_OPS || width == 0 || width > 256 || (w[0] >> 22) != 0u) {
            msg = "bad instruction " + std::to_string(i);   // bits 22..31 are the fused forms'
            return MG_EINVAL;
        }
        if (((w[0] >> 17) & 1u) && ((w[0] >> 18) & 0xfu) >= dags->n_slots) { msg = "slot out of range"; return MG_EINVAL; }
        if (op == BV_TAB) {
            const uint32_t imm = w[3], t = imm & 0xfffffu, lo = (imm >> 21) & 0xffu;
            if (t >= models->n_tables || (imm >> 29) != 0u || lo + width > 256u) {
                msg = "bad table reference at instruction " + std::to_string(i);
                return MG_EINVAL;
            }
        }
        const int nref = (op == BV_ITE) ? 3 : (op == BV_COPY || op == BV_NOT || op == BV_NEG || op == BV_BNOT ||
                                               op == BV_EXTRACT || op == BV_ZEXT || op == BV_SEXT) ? 1 : 2;
        for (int k = 0; k < nref; ++k) {
            const uint32_t ref = w[1 + k], kind = ref >> 30, idx = ref & 0x3fffffffu;
            if (k > 0 && kind == BV_REF_ACC) {
                msg = "accumulator operand past position A at instruction " + std::to_string(i);
                return MG_EINVAL;
            }
            if ((kind == BV_REF_SLOT && idx >= dags->n_slots) || (kind == BV_REF_VAR && idx >= models->n_vars) ||
                (kind == BV_REF_CONST && idx >= dags->n_consts)) {
                msg = "operand out of range at instruction " + std::to_string(i);
                return MG_EINVAL;
            }
        }
    }
    const char *fv = getenv("MG_BV_FUSE");
    const uint32_t *insns = dags->insns, *prog_off = dags->prog_off;
    uint32_t total_up = total;
    if (!(fv && fv[0] == '0')) {
        // superinstructions, all shapes (MG_BV_FUSE=0 uploads the programs as
        // given: the parity tests compare both; the per-shape A/B levels are in
        // ab/k2_fuse_levels.diff)
        bv_fuse(dags, s.h_insns, s.h_off, true, true, true, true);
    } else {
        s.h_insns.assign(dags->insns, dags->insns + 4 * (size_t)total);
        s.h_off.assign(dags->prog_off, dags->prog_off + n + 1);
    }
    bv_predecode(s.h_insns, s.h_off, n);
    insns = s.h_insns.data();
    prog_off = s.h_off.data();
    total_up = s.h_off[n];
    // tiles: consecutive DAGs whose programs fit BV_TILE_INSNS together
    // LDS tile capacity: the longest program rounded up, at least BV_TILE_MIN, so
    // short-program batches keep a small LDS footprint (higher occupancy)
    uint32_t longest = 0;
    for (uint32_t d = 0; d < n; ++d) longest = std::max(longest, prog_off[d + 1] - prog_off[d]);
    s.tile_cap = std::max<uint32_t>(BV_TILE_MIN, (longest + 255u) & ~255u);
    s.h_tiles.clear();
    s.h_tiles.push_back(0);
    uint32_t acc = 0;
    for (uint32_t d = 0; d < n; ++d) {
        const uint32_t len = prog_off[d + 1] - prog_off[d];
        if (acc + len > s.tile_cap || (d - s.h_tiles.back()) >= BV_TILE_DAGS) { s.h_tiles.push_back(d); acc = 0; }
        acc += len;
    }
    s.h_tiles.push_back(n);
    s.n_tiles = (uint32_t)s.h_tiles.size() - 1;
    int rc = 0;
    if ((rc = bv_ensure(s.insns, s.cap_insns, total_up))) { msg = "alloc insns"; return rc; }
    if ((rc = bv_ensure(s.prog_off, s.cap_dags, (size_t)n + 1))) { msg = "alloc offsets"; return rc; }
    if ((rc = bv_ensure(s.tile_dag, s.cap_tiles, s.h_tiles.size()))) { msg = "alloc tiles"; return rc; }
    if ((rc = bv_ensure(s.consts, s.cap_consts, (size_t)std::max<uint32_t>(dags->n_consts, 1) * 2))) { msg = "alloc consts"; return rc; }
    if ((rc = bv_ensure(s.values, s.cap_values, (size_t)std::max<uint32_t>(models->n_vars, 1) * models->n_models * 2))) { msg = "alloc values"; return rc; }
    if (models->n_tables) {
        if (!models->tab_start || !models->tab_count || !models->tab_default ||
            (models->n_entries && !models->tab_entries)) { msg = "table arrays missing"; return MG_EINVAL; }
        const size_t tm = (size_t)models->n_tables * models->n_models;
        for (size_t k = 0; k < tm; ++k)
            if ((uint64_t)models->tab_start[k] + models->tab_count[k] > models->n_entries) {
                msg = "table entries out of range"; return MG_EINVAL;
            }
        hipFree(s.tab_start); hipFree(s.tab_count); hipFree(s.tab_default);
        s.tab_start = s.tab_count = nullptr;
        s.tab_default = nullptr;
        if (hipMalloc(&s.tab_start, tm * 4) != hipSuccess || hipMalloc(&s.tab_count, tm * 4) != hipSuccess ||
            hipMalloc(&s.tab_default, tm * 64) != hipSuccess) {
            msg = "alloc tables"; return MG_ENOMEM;
        }
        if ((rc = bv_ensure(s.tab_entries, s.cap_entries, (size_t)std::max<uint32_t>(models->n_entries, 1) * 8))) {
            msg = "alloc table entries"; return rc;
        }
    }
    hipFree(s.first_sat); hipFree(s.sat_count);
    s.first_sat = s.sat_count = nullptr;
    if (hipMalloc(&s.first_sat, (size_t)n * 4) != hipSuccess || hipMalloc(&s.sat_count, (size_t)n * 4) != hipSuccess) {
        msg = "alloc outputs";
        return MG_ENOMEM;
    }
    hipError_t e = hipSuccess;
    e = e ? e : hipMemcpyAsync(s.insns, insns, (size_t)total_up * 16, hipMemcpyHostToDevice, st);
    e = e ? e : hipMemcpyAsync(s.prog_off, prog_off, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, st);
    e = e ? e : hipMemcpyAsync(s.tile_dag, s.h_tiles.data(), s.h_tiles.size() * 4, hipMemcpyHostToDevice, st);
    if (dags->n_consts) e = e ? e : hipMemcpyAsync(s.consts, dags->consts, (size_t)dags->n_consts * 32, hipMemcpyHostToDevice, st);
    if (models->n_vars)
        e = e ? e : hipMemcpyAsync(s.values, models->values, (size_t)models->n_vars * models->n_models * 32, hipMemcpyHostToDevice, st);
    if (models->n_tables) {
        const size_t tm = (size_t)models->n_tables * models->n_models;
        e = e ? e : hipMemcpyAsync(s.tab_start, models->tab_start, tm * 4, hipMemcpyHostToDevice, st);
        e = e ? e : hipMemcpyAsync(s.tab_count, models->tab_count, tm * 4, hipMemcpyHostToDevice, st);
        e = e ? e : hipMemcpyAsync(s.tab_default, models->tab_default, tm * 64, hipMemcpyHostToDevice, st);
        if (models->n_entries)
            e = e ? e : hipMemcpyAsync(s.tab_entries, models->tab_entries, (size_t)models->n_entries * 128,
                                       hipMemcpyHostToDevice, st);
    }
    e = e ? e : hipStreamSynchronize(st);
    if (e != hipSuccess) { msg = std::string("bv upload: ") + hipGetErrorString(e); return MG_EDEVICE; }
    s.n_tables = models->n_tables; s.n_entries = models->n_entries;
    s.n_dags = n; s.n_models = models->n_models; s.n_vars = models->n_vars;
    s.n_slots = std::max<uint32_t>(dags->n_slots, 1); s.n_consts = dags->n_consts;
    return 0;
}

static int bv_run(BvState &s, uint32_t dag_first, uint32_t dag_count, hipStream_t st, std::string &msg) {
    if (!s.n_dags) { msg = "mg_eval_run before mg_eval_upload"; return MG_ESTATE; }
    if (dag_first + (uint64_t)dag_count > s.n_dags || dag_count == 0) { msg = "DAG range out of bounds"; return MG_EINVAL; }
    const uint32_t dag_hi = dag_first + dag_count;
    hipError_t e = hipMemsetAsync(s.first_sat + dag_first, 0xff, (size_t)dag_count * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(s.sat_count + dag_first, 0, (size_t)dag_count * 4, st);
    const uint32_t bit_words = (s.n_models + 63u) / 64u;
    if (s.want_bits) {
        const size_t need = (size_t)s.n_dags * bit_words;
        if (bv_ensure(s.sat_bits, s.cap_bits, need)) { msg = "alloc sat bitmap"; return MG_ENOMEM; }
        if (e == hipSuccess)
            e = hipMemsetAsync(s.sat_bits + (size_t)dag_first * bit_words, 0, (size_t)dag_count * bit_words * 8, st);
    }
    if (e != hipSuccess) { msg = hipGetErrorString(e); return MG_EDEVICE; }
    // tiles covering [dag_first, dag_hi)
    const auto &t = s.h_tiles;
    uint32_t t0 = (uint32_t)(std::upper_bound(t.begin(), t.end(), dag_first) - t.begin()) - 1;
    uint32_t t1 = (uint32_t)(std::lower_bound(t.begin(), t.end(), dag_hi) - t.begin());
    const uint32_t nt = t1 - t0;
    const uint32_t tiles_pad = (nt + 7u) & ~7u;
    // model chunks per block: as many as keep >= BV_GROUP_TARGET blocks in flight,
    // so each program tile is staged once per block instead of once per chunk
    const uint32_t chunk_models = BV_BLOCK;
    const uint32_t chunks = (s.n_models + chunk_models - 1) / chunk_models;
    const uint32_t groups_wanted = std::max<uint32_t>(1u, (BV_GROUP_TARGET + tiles_pad - 1u) / tiles_pad);
    const uint32_t cpb = std::max<uint32_t>(1u, chunks / std::min(groups_wanted, chunks));
    const uint32_t groups = (chunks + cpb - 1u) / cpb;
    const size_t grid = (size_t)tiles_pad * groups;
    if (grid > 0x7fffffffull) { msg = "grid too large"; return MG_EINVAL; }
    const size_t lds = (size_t)s.n_slots * 2 * BV_BLOCK * sizeof(uint4);
    static bool lds_attr = false;      // programs with more than 4 slots need > 64 KiB of LDS
    if (!lds_attr) {
        (void)hipFuncSetAttribute((const void *)k_bv_eval, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(BV_MAX_SLOTS * 2 * BV_BLOCK * sizeof(uint4)));
        lds_attr = true;
    }
    hipLaunchKernelGGL(k_bv_eval, dim3((unsigned)grid), dim3(BV_BLOCK), lds, st,
                       s.insns, s.prog_off, s.tile_dag,
                       s.consts, s.values, s.n_models, BvTables{s.tab_start, s.tab_count, s.tab_entries, s.tab_default},
                       s.n_slots, t0, nt, tiles_pad, dag_first, dag_hi,
                       s.tile_cap, cpb, s.first_sat, s.sat_count, s.want_bits ? s.sat_bits : nullptr, bit_words);
    e = hipGetLastError();
    if (e != hipSuccess) { msg = std::string("k_bv_eval launch: ") + hipGetErrorString(e); return MG_EDEVICE; }
    return 0;
}

static int bv_download(BvState &s, uint32_t *first_sat, uint32_t *sat_count, uint32_t dag_first, uint32_t dag_count,
                       hipStream_t st, std::string &msg, unsigned long long *sat_bits = nullptr) {
    if (dag_first + (uint64_t)dag_count > s.n_dags) { msg = "DAG range out of bounds"; return MG_EINVAL; }
    hipError_t e = hipSuccess;
    if (sat_bits) {
        if (!s.want_bits || !s.sat_bits) { msg = "no bitmap was computed"; return MG_ESTATE; }
        const size_t bw = (s.n_models + 63u) / 64u;
        e = hipMemcpyAsync(sat_bits, s.sat_bits + (size_t)dag_first * bw, (size_t)dag_count * bw * 8,
                           hipMemcpyDeviceToHost, st);
    }
    if (first_sat) e = hipMemcpyAsync(first_sat, s.first_sat + dag_first, (size_t)dag_count * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && sat_count)
        e = hipMemcpyAsync(sat_count, s.sat_count + dag_first, (size_t)dag_count * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) { msg = hipGetErrorString(e); return MG_EDEVICE; }
    return 0;
}
