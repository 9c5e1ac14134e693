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
    BV_NUM_OPS
};

#define BV_REF_ACC 0u
#define BV_REF_SLOT 1u
#define BV_REF_VAR 2u
#define BV_REF_CONST 3u
#define BV_MAX_SLOTS 8u
#define BV_BLOCK 256u
#define BV_TILE_INSNS 2048u   // longest program (LDS tile upper bound: 32 KiB)
#define BV_TILE_MIN 512u      // smallest LDS tile (8 KiB)
#define BV_TILE_DAGS 64u      // most DAGs per tile (per-block result accumulators)
#define BV_GROUP_TARGET 4096u // blocks wanted per launch (16 per CU)
#define BV_MPT_DEFAULT 2u     // models per thread (k_bv_eval<.., M>)
#define BV_LDS_MAX (96u * 1024u)   // dynamic LDS a kernel-2 block may take

struct BvState {
    uint32_t n_dags = 0, n_models = 0, n_vars = 0, n_slots = 0, n_consts = 0, n_tiles = 0, tile_cap = 0;
    uint4 *timg = nullptr;           // tile images: per tile [its instructions][its constants x 2]
    uint32_t *prog_off = nullptr;    // [n_dags + 1] instruction offsets (global numbering)
    uint32_t *tile_dag = nullptr;    // [n_tiles + 1] first DAG of each tile
    uint32_t *tile_img = nullptr;    // [n_tiles + 1] offset (uint4) of each tile image in timg
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
    size_t cap_timg = 0, cap_dags = 0, cap_values = 0, cap_tiles = 0, cap_timgoff = 0;
    size_t cap_entries = 0;
    uint32_t mpt = BV_MPT_DEFAULT;   // models per thread (1, 2 or 4); MG_BV_MPT overrides
    std::vector<uint32_t> h_tiles, h_timg_off;
    std::vector<uint4> h_timg;
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

struct BvCtx {
    const uint4 *__restrict__ values;
    const uint4 *consts;   // LDS: this tile's constants (2 x uint4 each)
    uint4 *slots;          // LDS [n_slots][2][M][BV_BLOCK]
    uint32_t n_models, tid;
    BvTables tab;
};

DEV U256 ld2(const uint4 *p) {
    const uint4 x = p[0], y = p[1];
    U256 r;
    r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
    r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
    return r;
}

// model interpretation lookup (entries are unique keys: first match wins)
DEV U256 bv_table(BvTables tab, uint32_t n_models, uint32_t model, U256 k0, U256 k1,
                                      uint32_t imm) {
    const uint32_t t = imm & 0xfffffu, part = (imm >> 20) & 1u, lo = (imm >> 21) & 0xffu;
    const size_t tm = (size_t)t * n_models + model;
    const uint32_t s0 = tab.start[tm], cnt = tab.count[tm];
    U256 v = ld2(tab.dflt + tm * 4u + part * 2u);
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint4 *e = tab.entries + (size_t)(s0 + k) * 8u;
        if (u_eq(ld2(e), k0) && u_eq(ld2(e + 2), k1)) {
            v = ld2(e + 4 + part * 2u);
            break;
        }
    }
    return lo ? u_shr_n(v, lo, 0u) : v;
}

// division-class ops (z3 semantics, division by zero included)
DEV U256 bv_divop(uint32_t op, U256 A, U256 B, uint32_t width, uint32_t rc) {
    switch (op) {
    case BV_UDIV: return z_udiv(A, B);
    case BV_UREM: return z_urem(A, B);
    case BV_SDIV: return z_sdiv(bv_sext(A, width), bv_sext(B, width));
    case BV_SREM: return z_srem(bv_sext(A, width), bv_sext(B, width));
    case BV_SMOD: return z_smod(bv_sext(A, width), bv_sext(B, width));
    default: {                     // BV_MUL_NOOVF_U: high w bits of the 2w-bit product are 0
        bool ovf;
        if (u_iszero(A) || u_iszero(B)) ovf = false;
        else {
            const U256 q = z_udiv(bv_mask(u_ones(), rc), A);
            ovf = u_lt(q, B);      // a*b > 2^w - 1  <=>  b > floor((2^w-1)/a)
        }
        return u_small(!ovf);
    }
    }
}

// M models per thread: thread t of a block evaluates models
// chunk_base + m * BV_BLOCK + t (m < M) with ONE instruction stream, so the
// instruction fetch, decode and dispatch (scalar, wave-uniform) are paid once
// for M evaluations.
template <int M>
DEV void bv_fetch(const BvCtx &c, const U256 (&acc)[M], uint32_t ref, const uint32_t (&model)[M],
                  U256 (&out)[M]) {
    const uint32_t kind = ref >> 30, idx = ref & 0x3fffffffu;
    if (kind == BV_REF_ACC) {
#pragma unroll
        for (int m = 0; m < M; ++m) out[m] = acc[m];
    } else if (kind == BV_REF_SLOT) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const uint4 x = c.slots[((idx * 2u) * M + m) * BV_BLOCK + c.tid];
            const uint4 y = c.slots[((idx * 2u + 1u) * M + m) * BV_BLOCK + c.tid];
            out[m].w[0] = x.x; out[m].w[1] = x.y; out[m].w[2] = x.z; out[m].w[3] = x.w;
            out[m].w[4] = y.x; out[m].w[5] = y.y; out[m].w[6] = y.z; out[m].w[7] = y.w;
        }
    } else if (kind == BV_REF_VAR) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const size_t row = (size_t)idx * c.n_models + model[m];
            const uint4 x = c.values[2 * row], y = c.values[2 * row + 1];
            out[m].w[0] = x.x; out[m].w[1] = x.y; out[m].w[2] = x.z; out[m].w[3] = x.w;
            out[m].w[4] = y.x; out[m].w[5] = y.y; out[m].w[6] = y.z; out[m].w[7] = y.w;
        }
    } else {
        // constant: the tile's own pool, staged in LDS with its instructions
        // (uniform address: a broadcast read), shared by the M models
        const uint4 x = c.consts[2u * idx], y = c.consts[2u * idx + 1u];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            out[m].w[0] = x.x; out[m].w[1] = x.y; out[m].w[2] = x.z; out[m].w[3] = x.w;
            out[m].w[4] = y.x; out[m].w[5] = y.y; out[m].w[6] = y.z; out[m].w[7] = y.w;
        }
    }
}

#define BV_FOR_M _Pragma("unroll") for (int m = 0; m < M; ++m)

// Apply a large op (Knuth division, table scan) to the M models with ONE inlined
// copy of its code: a rolled loop over m whose operands and result move through
// static-index selects on the (uniform) loop counter, so nothing is dynamically
// indexed (no scratch) and the code is not replicated M times.
#define BV_ROLLED(EXPR)                                                        \
    do {                                                                       \
        if (M == 1) {                                                          \
            const U256 a_ = A[0], b_ = B[0];                                   \
            const uint32_t model_ = model[0];                                  \
            r[0] = (EXPR);                                                     \
            break;                                                             \
        }                                                                      \
        _Pragma("nounroll") for (int mm = 0; mm < M; ++mm) {                   \
            U256 a_ = A[0], b_ = B[0];                                         \
            uint32_t model_ = model[0];                                        \
            _Pragma("unroll") for (int k = 1; k < M; ++k)                      \
                if (k == mm) { a_ = A[k]; b_ = B[k]; model_ = model[k]; }      \
            const U256 res_ = (EXPR);                                          \
            _Pragma("unroll") for (int k = 0; k < M; ++k)                      \
                if (k == mm) r[k] = res_;                                      \
        }                                                                      \
    } while (0)

template <int M>
__global__ __launch_bounds__(BV_BLOCK) void k_bv_eval(const uint4 *__restrict__ timg,
                                                      const uint32_t *__restrict__ prog_off,
                                                      const uint32_t *__restrict__ tile_dag,
                                                      const uint32_t *__restrict__ tile_img,
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
    // The tile image — the tile's programs followed by the constants they use,
    // remapped to tile-local indices on the host (bv_upload) — is staged into LDS
    // with one coalesced copy and read with broadcast ds_reads; constants never
    // cost a dependent scalar load from a table that, at C4's 1M DAGs, is 1 GB.
    uint4 *prog = smem;                          // [tile_cap]
    uint4 *slots = smem + tile_cap;              // [n_slots][2][M][BV_BLOCK]
    // group-major order with the tile count padded to a multiple of 8: the blocks
    // of one program tile share blockIdx % 8, i.e. one XCD's L2 (speed only)
    const uint32_t b = blockIdx.x;
    const uint32_t tile = tile_first + (b % tiles_pad);
    const uint32_t group = b / tiles_pad;
    if (tile >= tile_first + n_tiles) return;
    const uint32_t d0 = max(tile_dag[tile], dag_lo), d1 = min(tile_dag[tile + 1], dag_hi);
    if (d0 >= d1) return;
    // the tile is read from HBM once per block and reused for every model chunk
    // per-block results of the tile's DAGs: waves combine in LDS, the block adds
    // its totals to HBM once per DAG (not one atomic pair per wave per DAG)
    __shared__ uint32_t blk_cnt[BV_TILE_DAGS], blk_first[BV_TILE_DAGS];
    if (threadIdx.x < BV_TILE_DAGS) { blk_cnt[threadIdx.x] = 0u; blk_first[threadIdx.x] = 0xffffffffu; }
    const uint32_t img0 = tile_img[tile], img_n = tile_img[tile + 1] - img0;
    // a range-limited run (dag_lo/dag_hi) stages the whole tile: consts follow
    // the tile's full instruction list
    const uint32_t t_i0 = prog_off[tile_dag[tile]], t_n = prog_off[tile_dag[tile + 1]] - t_i0;
    for (uint32_t i = threadIdx.x; i < img_n; i += BV_BLOCK) prog[i] = timg[img0 + i];
    __syncthreads();
    const uint4 *tconst = prog + t_n;

    const uint32_t tid = threadIdx.x;
    constexpr uint32_t CHUNK = BV_BLOCK * (uint32_t)M;
    const uint32_t n_chunks = (n_models + CHUNK - 1u) / CHUNK;
    const uint32_t c_lo = group * chunks_per_block, c_hi = min(c_lo + chunks_per_block, n_chunks);
    for (uint32_t chunk = c_lo; chunk < c_hi; ++chunk) {
    uint32_t model[M];
    bool live[M];
    BV_FOR_M {
        const uint32_t mm = chunk * CHUNK + (uint32_t)m * BV_BLOCK + tid;
        live[m] = mm < n_models;
        model[m] = live[m] ? mm : 0u;
    }
    const BvCtx c{values, tconst, slots, n_models, tid, tab};

    for (uint32_t d = d0; d < d1; ++d) {
        const uint32_t p0 = prog_off[d] - t_i0, p1 = prog_off[d + 1] - t_i0;
        U256 acc[M];
        BV_FOR_M acc[m] = u_zero();
        for (uint32_t p = p0; p < p1; ++p) {
            const uint4 ins = prog[p];
            const uint32_t w0 = uni(ins.x), ra = uni(ins.y), rb = uni(ins.z), rc = uni(ins.w);
            const uint32_t op = w0 & 0xffu, width = (w0 >> 8) & 0x1ffu;
            U256 A[M], r[M];
            bv_fetch<M>(c, acc, ra, model, A);
            switch (op) {
            case BV_COPY: BV_FOR_M r[m] = A[m]; break;
            case BV_NOT: BV_FOR_M r[m] = u_not(A[m]); break;
            case BV_NEG: BV_FOR_M r[m] = u_neg(A[m]); break;
            case BV_BNOT: BV_FOR_M r[m] = u_small((A[m].w[0] & 1u) ^ 1u); break;
            case BV_EXTRACT: BV_FOR_M r[m] = u_shr_n(A[m], rb & 0xffu, 0u); break;
            case BV_ZEXT: BV_FOR_M r[m] = A[m]; break;
            case BV_SEXT: BV_FOR_M r[m] = bv_sext(A[m], rb); break;
            default: {
                U256 B[M];
                bv_fetch<M>(c, acc, rb, model, B);
                switch (op) {
                case BV_ADD: BV_FOR_M r[m] = u_add(A[m], B[m]); break;
                case BV_SUB: BV_FOR_M r[m] = u_sub(A[m], B[m]); break;
                case BV_MUL: BV_FOR_M r[m] = u_mul(A[m], B[m]); break;
                case BV_UDIV: case BV_UREM: case BV_SDIV: case BV_SREM: case BV_SMOD: case BV_MUL_NOOVF_U:
                    BV_ROLLED(bv_divop(op, a_, b_, width, rc));
                    break;
                case BV_AND: BV_FOR_M r[m] = u_and(A[m], B[m]); break;
                case BV_OR: BV_FOR_M r[m] = u_or(A[m], B[m]); break;
                case BV_XOR: BV_FOR_M r[m] = u_xor(A[m], B[m]); break;
                case BV_SHL:
                    BV_FOR_M r[m] = (u_fits32(B[m]) && B[m].w[0] < width) ? u_shl_n(A[m], B[m].w[0]) : u_zero();
                    break;
                case BV_LSHR:
                    BV_FOR_M r[m] = (u_fits32(B[m]) && B[m].w[0] < width) ? u_shr_n(A[m], B[m].w[0], 0u) : u_zero();
                    break;
                case BV_ASHR:
                    BV_FOR_M {
                        const U256 sa = bv_sext(A[m], width);
                        const uint32_t fill = u_isneg(sa) ? 0xffffffffu : 0u;
                        const uint32_t sh = (u_fits32(B[m]) && B[m].w[0] < width) ? B[m].w[0] : 255u;
                        r[m] = u_shr_n(sa, sh, fill);
                    }
                    break;
                case BV_EQ: BV_FOR_M r[m] = u_small(u_eq(A[m], B[m])); break;
                case BV_NE: BV_FOR_M r[m] = u_small(!u_eq(A[m], B[m])); break;
                case BV_ULT: BV_FOR_M r[m] = u_small(u_lt(A[m], B[m])); break;
                case BV_ULE: BV_FOR_M r[m] = u_small(!u_lt(B[m], A[m])); break;
                case BV_UGT: BV_FOR_M r[m] = u_small(u_lt(B[m], A[m])); break;
                case BV_UGE: BV_FOR_M r[m] = u_small(!u_lt(A[m], B[m])); break;
                case BV_SLT: BV_FOR_M r[m] = u_small(u_slt(bv_sext(A[m], rc), bv_sext(B[m], rc))); break;
                case BV_SLE: BV_FOR_M r[m] = u_small(!u_slt(bv_sext(B[m], rc), bv_sext(A[m], rc))); break;
                case BV_SGT: BV_FOR_M r[m] = u_small(u_slt(bv_sext(B[m], rc), bv_sext(A[m], rc))); break;
                case BV_SGE: BV_FOR_M r[m] = u_small(!u_slt(bv_sext(A[m], rc), bv_sext(B[m], rc))); break;
                case BV_BAND: BV_FOR_M r[m] = u_small(A[m].w[0] & B[m].w[0] & 1u); break;
                case BV_BOR: BV_FOR_M r[m] = u_small((A[m].w[0] | B[m].w[0]) & 1u); break;
                case BV_BXOR: BV_FOR_M r[m] = u_small((A[m].w[0] ^ B[m].w[0]) & 1u); break;
                case BV_BIMPLIES: BV_FOR_M r[m] = u_small(((A[m].w[0] & 1u) ^ 1u) | (B[m].w[0] & 1u)); break;
                case BV_ITE: {
                    U256 C[M];
                    bv_fetch<M>(c, acc, rc, model, C);
                    BV_FOR_M r[m] = u_select((A[m].w[0] & 1u) != 0u, B[m], C[m]);
                    break;
                }
                case BV_CONCAT: BV_FOR_M r[m] = u_or(u_shl_n(A[m], rc), B[m]); break;
                case BV_ADD_NOOVF_U:   // top bit of the (w+1)-bit sum is 0
                    BV_FOR_M {
                        const U256 s = u_add(A[m], B[m]);
                        const bool ovf = rc >= 256u ? u_lt(s, A[m]) : !u_iszero(u_shr_n(s, rc, 0u));
                        r[m] = u_small(!ovf);
                    }
                    break;
                case BV_SUB_NOUDF_U: BV_FOR_M r[m] = u_small(!u_lt(A[m], B[m])); break;
                case BV_TAB: BV_ROLLED(bv_table(c.tab, n_models, model_, a_, b_, rc)); break;
                default: BV_FOR_M r[m] = u_zero(); break;
                }
            }
            }
            if (width < 256u) { BV_FOR_M r[m] = bv_mask(r[m], width); }
            BV_FOR_M acc[m] = r[m];
            if ((w0 >> 17) & 1u) {
                const uint32_t ds = (w0 >> 18) & 0xfu;
                BV_FOR_M {
                    slots[((ds * 2u) * M + m) * BV_BLOCK + tid] = make_uint4(r[m].w[0], r[m].w[1], r[m].w[2], r[m].w[3]);
                    slots[((ds * 2u + 1u) * M + m) * BV_BLOCK + tid] = make_uint4(r[m].w[4], r[m].w[5], r[m].w[6], r[m].w[7]);
                }
            }
        }
        BV_FOR_M {
            const bool sat = live[m] && (acc[m].w[0] & 1u);
            const uint64_t bal = __ballot(sat);
            if ((tid & 63u) == 0u && bal) {
                const uint32_t base = chunk * CHUNK + (uint32_t)m * BV_BLOCK + tid;   // tid % 64 == 0
                // optional per-model bitmap (one u64 per wave): lets the host replay
                // sequential check_quick_sat calls whose LRU bumps reorder the pool
                if (sat_bits) sat_bits[(size_t)d * bit_words + (base >> 6)] = bal;
                atomicAdd(&blk_cnt[d - d0], (uint32_t)__popcll(bal));
                atomicMin(&blk_first[d - d0], base + (uint32_t)(__ffsll((long long)bal) - 1));
            }
        }
    }
    }
    __syncthreads();
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
    hipFree(s.timg); hipFree(s.prog_off); hipFree(s.tile_dag); hipFree(s.tile_img);
    hipFree(s.values); hipFree(s.first_sat); hipFree(s.sat_count);
    hipFree(s.tab_start); hipFree(s.tab_count); hipFree(s.tab_entries); hipFree(s.tab_default);
    hipFree(s.sat_bits);
    s = BvState{};
}

static int bv_upload(BvState &s, const mg_dag_batch *dags, const mg_model_batch *models, hipStream_t st,
                     std::string &msg) {
    if (dags->n_dags == 0 || !dags->prog_off || !dags->insns) { msg = "empty DAG batch"; return MG_EINVAL; }
    if (dags->n_slots > BV_MAX_SLOTS) { msg = "too many slots"; return MG_EINVAL; }
    if (models->n_models == 0 || (models->n_vars && !models->values)) { msg = "empty model batch"; return MG_EINVAL; }
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
        if (op >= BV_NUM_OPS || width == 0 || width > 256) { msg = "bad instruction " + std::to_string(i); return MG_EINVAL; }
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
            if ((kind == BV_REF_SLOT && idx >= dags->n_slots) || (kind == BV_REF_VAR && idx >= models->n_vars) ||
                (kind == BV_REF_CONST && idx >= dags->n_consts)) {
                msg = "operand out of range at instruction " + std::to_string(i);
                return MG_EINVAL;
            }
        }
    }
    // Tiles: consecutive DAGs (at most BV_TILE_DAGS) whose tile image fits the LDS
    // tile: their instructions plus every constant they use, each constant once
    // per tile, operand refs rewritten to tile-local constant indices.
    const size_t slots_b1 = (size_t)std::max<uint32_t>(dags->n_slots, 1) * 2u * BV_BLOCK * sizeof(uint4);
    const uint32_t img_max = (uint32_t)((BV_LDS_MAX - slots_b1) / sizeof(uint4));
    auto nrefs = [](uint32_t op) -> int {
        return (op == BV_ITE) ? 3 : (op == BV_COPY || op == BV_NOT || op == BV_NEG || op == BV_BNOT ||
                                      op == BV_EXTRACT || op == BV_ZEXT || op == BV_SEXT) ? 1 : 2;
    };
    std::vector<uint32_t> stamp(std::max<uint32_t>(dags->n_consts, 1), 0xffffffffu);
    std::vector<uint32_t> local(std::max<uint32_t>(dags->n_consts, 1), 0u);
    // per DAG: its own distinct constants (image size alone) -> tile capacity
    uint32_t longest = 0;
    for (uint32_t d = 0; d < n; ++d) {
        uint32_t uc = 0;
        for (uint32_t i = dags->prog_off[d]; i < dags->prog_off[d + 1]; ++i) {
            const uint32_t *w = dags->insns + 4 * (size_t)i;
            for (int k = 0; k < nrefs(w[0] & 0xffu); ++k)
                if ((w[1 + k] >> 30) == BV_REF_CONST) {
                    const uint32_t g = w[1 + k] & 0x3fffffffu;
                    if (stamp[g] != d) { stamp[g] = d; ++uc; }
                }
        }
        longest = std::max(longest, dags->prog_off[d + 1] - dags->prog_off[d] + 2u * uc);
    }
    if (longest > img_max) { msg = "program plus its constants exceed the LDS tile"; return MG_EINVAL; }
    s.tile_cap = std::min(img_max, std::max<uint32_t>(BV_TILE_MIN, (longest + 255u) & ~255u));
    std::fill(stamp.begin(), stamp.end(), 0xffffffffu);
    s.h_tiles.assign(1, 0u);
    s.h_timg_off.assign(1, 0u);
    s.h_timg.clear();
    s.h_timg.reserve((size_t)total * 2);
    std::vector<uint32_t> tconsts;          // global indices of the current tile's constants
    uint32_t tile_id = 0, t_insns = 0;
    auto close_tile = [&](uint32_t d_end) {
        for (uint32_t g : tconsts) {
            const uint32_t *c = dags->consts + 8 * (size_t)g;
            s.h_timg.push_back(make_uint4(c[0], c[1], c[2], c[3]));
            s.h_timg.push_back(make_uint4(c[4], c[5], c[6], c[7]));
        }
        s.h_tiles.push_back(d_end);
        s.h_timg_off.push_back((uint32_t)s.h_timg.size());
        tconsts.clear();
        t_insns = 0;
        ++tile_id;
    };
    for (uint32_t d = 0; d < n; ++d) {
        const uint32_t a = dags->prog_off[d], b = dags->prog_off[d + 1];
        uint32_t fresh = 0;                 // constants this DAG adds to the tile
        for (uint32_t i = a; i < b; ++i) {
            const uint32_t *w = dags->insns + 4 * (size_t)i;
            for (int k = 0; k < nrefs(w[0] & 0xffu); ++k)
                if ((w[1 + k] >> 30) == BV_REF_CONST) {
                    const uint32_t g = w[1 + k] & 0x3fffffffu;
                    if (stamp[g] != tile_id && local[g] != 0xfffffffeu) { local[g] = 0xfffffffeu; ++fresh; }
                }
        }
        for (uint32_t i = a; i < b; ++i) {          // undo the counting marks
            const uint32_t *w = dags->insns + 4 * (size_t)i;
            for (int k = 0; k < nrefs(w[0] & 0xffu); ++k)
                if ((w[1 + k] >> 30) == BV_REF_CONST && local[w[1 + k] & 0x3fffffffu] == 0xfffffffeu)
                    local[w[1 + k] & 0x3fffffffu] = 0u;
        }
        if (d > s.h_tiles.back() &&
            (t_insns + (b - a) + 2u * ((uint32_t)tconsts.size() + fresh) > s.tile_cap ||
             d - s.h_tiles.back() >= BV_TILE_DAGS)) {
            close_tile(d);
            // the new tile's image starts with this DAG: instructions come first,
            // so move nothing -- images are built tile by tile below
        }
        for (uint32_t i = a; i < b; ++i) {
            const uint32_t *w = dags->insns + 4 * (size_t)i;
            uint32_t x[4] = {w[0], w[1], w[2], w[3]};
            for (int k = 0; k < nrefs(w[0] & 0xffu); ++k)
                if ((x[1 + k] >> 30) == BV_REF_CONST) {
                    const uint32_t g = x[1 + k] & 0x3fffffffu;
                    if (stamp[g] != tile_id) {
                        stamp[g] = tile_id;
                        local[g] = (uint32_t)tconsts.size();
                        tconsts.push_back(g);
                    }
                    x[1 + k] = (BV_REF_CONST << 30) | local[g];
                }
            s.h_timg.push_back(make_uint4(x[0], x[1], x[2], x[3]));
        }
        t_insns += b - a;
    }
    close_tile(n);
    s.h_tiles.pop_back();                         // close_tile pushed n: keep one n at the end
    s.h_tiles.push_back(n);
    s.n_tiles = (uint32_t)s.h_tiles.size() - 1;
    int rc = 0;
    if ((rc = bv_ensure(s.timg, s.cap_timg, s.h_timg.size()))) { msg = "alloc tile images"; return rc; }
    if ((rc = bv_ensure(s.prog_off, s.cap_dags, (size_t)n + 1))) { msg = "alloc offsets"; return rc; }
    if ((rc = bv_ensure(s.tile_dag, s.cap_tiles, s.h_tiles.size()))) { msg = "alloc tiles"; return rc; }
    if ((rc = bv_ensure(s.tile_img, s.cap_timgoff, s.h_timg_off.size()))) { msg = "alloc tile offsets"; return rc; }
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
    e = e ? e : hipMemcpyAsync(s.timg, s.h_timg.data(), s.h_timg.size() * 16, hipMemcpyHostToDevice, st);
    e = e ? e : hipMemcpyAsync(s.prog_off, dags->prog_off, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, st);
    e = e ? e : hipMemcpyAsync(s.tile_dag, s.h_tiles.data(), s.h_tiles.size() * 4, hipMemcpyHostToDevice, st);
    e = e ? e : hipMemcpyAsync(s.tile_img, s.h_timg_off.data(), s.h_timg_off.size() * 4, hipMemcpyHostToDevice, st);
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
    const char *mv = getenv("MG_BV_MPT");
    s.mpt = mv ? (uint32_t)atoi(mv) : BV_MPT_DEFAULT;
    if (s.mpt != 1u && s.mpt != 2u && s.mpt != 4u) s.mpt = BV_MPT_DEFAULT;
    // a pool smaller than one block of threads gains nothing from more models per thread
    while (s.mpt > 1u && (size_t)models->n_models <= (size_t)BV_BLOCK * (s.mpt / 2u)) s.mpt /= 2u;
    // LDS per block (program tile + M register slots per thread) within BV_LDS_MAX
    const size_t slots_b = (size_t)std::max<uint32_t>(dags->n_slots, 1) * 2u * BV_BLOCK * sizeof(uint4);
    while (s.mpt > 1u && (size_t)s.tile_cap * sizeof(uint4) + slots_b * s.mpt > BV_LDS_MAX) s.mpt /= 2u;
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
    const uint32_t chunk_models = BV_BLOCK * s.mpt;
    const uint32_t chunks = (s.n_models + chunk_models - 1) / chunk_models;
    const uint32_t groups_wanted = std::max<uint32_t>(1u, (BV_GROUP_TARGET + tiles_pad - 1u) / tiles_pad);
    const uint32_t cpb = std::max<uint32_t>(1u, chunks / std::min(groups_wanted, chunks));
    const uint32_t groups = (chunks + cpb - 1u) / cpb;
    const size_t grid = (size_t)tiles_pad * groups;
    if (grid > 0x7fffffffull) { msg = "grid too large"; return MG_EINVAL; }
    const size_t lds = ((size_t)s.tile_cap + (size_t)s.n_slots * 2 * BV_BLOCK * s.mpt) * sizeof(uint4);
    auto kern = s.mpt == 4u ? k_bv_eval<4> : s.mpt == 2u ? k_bv_eval<2> : k_bv_eval<1>;
    if (lds > 65536u) {
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)BV_LDS_MAX);
        (void)hipGetLastError();
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(BV_BLOCK), lds, st,
                       s.timg, s.prog_off, s.tile_dag, s.tile_img,
                       s.values, s.n_models, BvTables{s.tab_start, s.tab_count, s.tab_entries, s.tab_default},
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
