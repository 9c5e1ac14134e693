// u256.cuh — 256-bit two's-complement arithmetic on 8 x u32 limbs for CDNA4.
//
// Every loop is fully unrolled over compile-time limb indices so values stay in
// VGPRs (a runtime-indexed register array would go to scratch); runtime shift
// amounts are applied with a 3-stage limb barrel shifter (v_cndmask per limb)
// followed by a funnel shift per limb (v_alignbit_b32).  Semantics are z3's bit-vector
// semantics used by mythril/laser/smt/bitvec.py (bvudiv x 0 = 2^256-1,
// bvurem x 0 = x, bvsdiv x 0 = x<0 ? 1 : -1, bvsrem x 0 = x).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

struct U256 {
    uint32_t w[8];  // w[0] = least significant limb
};

DEV U256 u_zero() {
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = 0u;
    return r;
}
DEV U256 u_ones() {
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = 0xffffffffu;
    return r;
}
DEV U256 u_small(uint64_t x) {
    U256 r = u_zero();
    r.w[0] = (uint32_t)x;
    r.w[1] = (uint32_t)(x >> 32);
    return r;
}
DEV bool u_iszero(const U256 &a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.w[i];
    return o == 0u;
}
// high 7 limbs zero: the value is a u32
DEV bool u_fits32(const U256 &a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 1; i < 8; ++i) o |= a.w[i];
    return o == 0u;
}
DEV bool u_eq(const U256 &a, const U256 &b) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.w[i] ^ b.w[i];
    return o == 0u;
}
// Carry chains use __builtin_addc / __builtin_subc, which lower to one
// v_add_co / v_addc_co (v_sub_co / v_subb_co) per limb; the equivalent 64-bit
// formulation costs 4-5x the VALU instructions (v_lshl_add_u64 + moves).
// unsigned a < b: borrow out of a - b
DEV bool u_lt(const U256 &a, const U256 &b) {
    unsigned br = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) (void)__builtin_subc(a.w[i], b.w[i], br, &br);
    return br != 0u;
}
DEV bool u_isneg(const U256 &a) { return (a.w[7] >> 31) != 0u; }
DEV bool u_slt(const U256 &a, const U256 &b) {
    bool na = u_isneg(a), nb = u_isneg(b);
    return na != nb ? na : u_lt(a, b);
}
DEV U256 u_add(const U256 &a, const U256 &b) {
    U256 r;
    unsigned c = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = __builtin_addc(a.w[i], b.w[i], c, &c);
    return r;
}
DEV U256 u_sub(const U256 &a, const U256 &b) {
    U256 r;
    unsigned br = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = __builtin_subc(a.w[i], b.w[i], br, &br);
    return r;
}
DEV U256 u_neg(const U256 &a) { return u_sub(u_zero(), a); }
// low 256 bits of a*b (schoolbook, 36 limb products: 28 v_mad_u64_u32 and
// 8 v_mul_lo_u32 for the products that only feed limb 7)
DEV U256 u_mul(const U256 &a, const U256 &b) {
    uint32_t r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t carry = 0u;
#pragma unroll
        for (int j = 0; i + j < 8; ++j) {
            if (i + j == 7) {
                r[7] += a.w[i] * b.w[j] + carry;
            } else {
                uint64_t t = (uint64_t)a.w[i] * b.w[j] + r[i + j];
                t += carry;
                r[i + j] = (uint32_t)t;
                carry = (uint32_t)(t >> 32);
            }
        }
    }
    U256 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o.w[i] = r[i];
    return o;
}
DEV U256 u_and(const U256 &a, const U256 &b) {
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = a.w[i] & b.w[i];
    return r;
}
DEV U256 u_or(const U256 &a, const U256 &b) {
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = a.w[i] | b.w[i];
    return r;
}
DEV U256 u_xor(const U256 &a, const U256 &b) {
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = a.w[i] ^ b.w[i];
    return r;
}
DEV U256 u_not(const U256 &a) {
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = ~a.w[i];
    return r;
}
DEV U256 u_select(bool c, const U256 &a, const U256 &b) {
    U256 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.w[i] = c ? a.w[i] : b.w[i];
    return r;
}

// ---- shifts ------------------------------------------------------------------
// limb barrel shifts by q in [0, 8)
DEV U256 u_shl_limbs(U256 a, uint32_t q) {
#pragma unroll
    for (int stage = 0; stage < 3; ++stage) {
        const int s = 1 << stage;
        const bool on = (q >> stage) & 1u;
        U256 t;
#pragma unroll
        for (int i = 0; i < 8; ++i) t.w[i] = i >= s ? a.w[i - s] : 0u;
        a = u_select(on, t, a);
    }
    return a;
}
DEV U256 u_shr_limbs(U256 a, uint32_t q, uint32_t fill) {
#pragma unroll
    for (int stage = 0; stage < 3; ++stage) {
        const int s = 1 << stage;
        const bool on = (q >> stage) & 1u;
        U256 t;
#pragma unroll
        for (int i = 0; i < 8; ++i) t.w[i] = i + s < 8 ? a.w[i + s] : fill;
        a = u_select(on, t, a);
    }
    return a;
}
// The same limb moves with each stage skipped when no lane of the wave needs it
// (one ballot each): in kernel 2's division the normalisation shift is below 32
// bits for nearly every lane (random 256-bit divisors), so the three 8-wide
// v_cndmask stages usually all drop out.
DEV U256 u_shl_limbs_w(U256 a, uint32_t q) {
#pragma unroll
    for (int stage = 0; stage < 3; ++stage) {
        const int s = 1 << stage;
        const bool on = (q >> stage) & 1u;
        if (__ballot(on) == 0ull) continue;
        U256 t;
#pragma unroll
        for (int i = 0; i < 8; ++i) t.w[i] = i >= s ? a.w[i - s] : 0u;
        a = u_select(on, t, a);
    }
    return a;
}
DEV U256 u_shr_limbs_w(U256 a, uint32_t q, uint32_t fill) {
#pragma unroll
    for (int stage = 0; stage < 3; ++stage) {
        const int s = 1 << stage;
        const bool on = (q >> stage) & 1u;
        if (__ballot(on) == 0ull) continue;
        U256 t;
#pragma unroll
        for (int i = 0; i < 8; ++i) t.w[i] = i + s < 8 ? a.w[i + s] : fill;
        a = u_select(on, t, a);
    }
    return a;
}
// (hi:lo) << r, high half, r in [0,32).  v_alignbit_b32 keeps each funnel
// shift in one VALU op; written as a 64-bit shift of (hi << 32 | lo) the
// compiler may merge adjacent limbs into 64-bit scratch loads instead.
DEV uint32_t fsl(uint32_t hi, uint32_t lo, uint32_t r) {
    return r == 0u ? hi : __builtin_amdgcn_alignbit(hi, lo, 32u - r);
}
// (hi:lo) >> r, low half, r in [0,32)
DEV uint32_t fsr(uint32_t hi, uint32_t lo, uint32_t r) {
    return __builtin_amdgcn_alignbit(hi, lo, r);
}
// a << n for n < 256
DEV U256 u_shl_n(U256 a, uint32_t n) {
    a = u_shl_limbs(a, n >> 5);
    const uint32_t r = n & 31u;
    U256 o;
#pragma unroll
    for (int i = 7; i >= 1; --i) o.w[i] = fsl(a.w[i], a.w[i - 1], r);
    o.w[0] = a.w[0] << r;
    return o;
}
// logical a >> n for n < 256; fill = 0 or 0xffffffff (arithmetic)
DEV U256 u_shr_n(U256 a, uint32_t n, uint32_t fill) {
    a = u_shr_limbs(a, n >> 5, fill);
    const uint32_t r = n & 31u;
    U256 o;
#pragma unroll
    for (int i = 0; i < 7; ++i) o.w[i] = fsr(a.w[i + 1], a.w[i], r);
    o.w[7] = fsr(fill, a.w[7], r);
    return o;
}
// u_shl_n / u_shr_n with the wave-skipped limb stages (kernel 2's division)
DEV U256 u_shl_n_w(U256 a, uint32_t n) {
    a = u_shl_limbs_w(a, n >> 5);
    const uint32_t r = n & 31u;
    U256 o;
#pragma unroll
    for (int i = 7; i >= 1; --i) o.w[i] = fsl(a.w[i], a.w[i - 1], r);
    o.w[0] = a.w[0] << r;
    return o;
}
DEV U256 u_shr_n_w(U256 a, uint32_t n, uint32_t fill) {
    a = u_shr_limbs_w(a, n >> 5, fill);
    const uint32_t r = n & 31u;
    U256 o;
#pragma unroll
    for (int i = 0; i < 7; ++i) o.w[i] = fsr(a.w[i + 1], a.w[i], r);
    o.w[7] = fsr(fill, a.w[7], r);
    return o;
}
// Shifts by a wave-uniform amount n < 256 (an instruction immediate, a constant
// operand): the limb move is a scalar branch over n / 32 with one static
// permutation per case (8 moves) instead of the three-stage v_cndmask barrel
// (24 VALU); the funnel shift is the same 8 v_alignbit.  n must be uniform
// across the wave (the caller guarantees it: the branches are scalar).
#define U_LIMB_CASES(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
DEV U256 u_shl_u(const U256 &a, uint32_t n) {
    U256 t;
    switch (n >> 5) {
#define U_SHL_CASE(Q) case Q: _Pragma("unroll") for (int i = 0; i < 8; ++i) t.w[i] = i >= Q ? a.w[i - Q] : 0u; break;
    U_LIMB_CASES(U_SHL_CASE)
#undef U_SHL_CASE
    default: t = u_zero(); break;
    }
    const uint32_t r = n & 31u;
    if (r == 0u) return t;
    U256 o;
#pragma unroll
    for (int i = 7; i >= 1; --i) o.w[i] = __builtin_amdgcn_alignbit(t.w[i], t.w[i - 1], 32u - r);
    o.w[0] = t.w[0] << r;
    return o;
}
// (a >> n) with `fill` shifted in (0, or 0xffffffff for an arithmetic shift)
DEV U256 u_shr_u(const U256 &a, uint32_t n, uint32_t fill) {
    U256 t;
    switch (n >> 5) {
#define U_SHR_CASE(Q) case Q: _Pragma("unroll") for (int i = 0; i < 8; ++i) t.w[i] = i + Q < 8 ? a.w[i + Q] : fill; break;
    U_LIMB_CASES(U_SHR_CASE)
#undef U_SHR_CASE
    default: t = u_zero(); break;
    }
    const uint32_t r = n & 31u;
    if (r == 0u) return t;
    U256 o;
#pragma unroll
    for (int i = 0; i < 7; ++i) o.w[i] = __builtin_amdgcn_alignbit(t.w[i + 1], t.w[i], r);
    o.w[7] = __builtin_amdgcn_alignbit(fill, t.w[7], r);
    return o;
}
#undef U_LIMB_CASES

// z3 bvshl / bvlshr / bvashr (shift >= 256 -> 0 / sign fill)
DEV U256 u_shl(const U256 &a, const U256 &s) {
    if (!u_fits32(s) || s.w[0] >= 256u) return u_zero();
    return u_shl_n(a, s.w[0]);
}
DEV U256 u_lshr(const U256 &a, const U256 &s) {
    if (!u_fits32(s) || s.w[0] >= 256u) return u_zero();
    return u_shr_n(a, s.w[0], 0u);
}
DEV U256 u_ashr(const U256 &a, const U256 &s) {
    const uint32_t fill = u_isneg(a) ? 0xffffffffu : 0u;
    if (!u_fits32(s) || s.w[0] >= 256u) {
        U256 r;
#pragma unroll
        for (int i = 0; i < 8; ++i) r.w[i] = fill;
        return r;
    }
    return u_shr_n(a, s.w[0], fill);
}
// number of significant bits (0 for 0)
DEV uint32_t u_bitlen(const U256 &a) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (a.w[i]) r = 32u * i + 32u - (uint32_t)__builtin_clz(a.w[i]);
    return r;
}
DEV uint32_t u_popcount(const U256 &a) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) p += (uint32_t)__builtin_popcount(a.w[i]);
    return p;
}

// ---- division ------------------------------------------------------------------
// Unsigned a / b and a % b for b != 0.
//
// * power-of-two divisors are shifts;
// * when every lane of the wave needs at most 32 quotient bits (bitlen(a) -
//   bitlen(b) < 32: selector extraction, comparisons of similar magnitudes) the
//   wave runs shift-subtract over only those bit positions;
// * otherwise Knuth's algorithm D on 32-bit digits: b is normalised so its top
//   bit is bit 255, a is shifted into 16 limbs by the same amount, and the 8
//   quotient digits come out top-down.  Each digit is estimated from the top two
//   remainder limbs with a Moller-Granlund 2-by-1 division by the precomputed
//   reciprocal of b's top limb (no per-digit hardware divide), refined against
//   the second limb, then the digit times b is subtracted with one add-back
//   when the estimate was still one too large.  All limb indices are static
//   (unrolled), so the 17-limb remainder stays in VGPRs.
DEV uint32_t mulhi32(uint32_t a, uint32_t b) { return __umulhi(a, b); }

// floor((2^64 - 1) / d) - 2^32 for d with its top bit set (MG 2011, eq. 1)
DEV uint32_t mg_reciprocal(uint32_t d) {
    return (uint32_t)((((uint64_t)(~d) << 32) | 0xffffffffull) / d);
}
// The same from the correctly rounded fp64 quotient 2^64 / d (absolute error < 2^-19),
// made exact against the defining inequality (2^32 + v) d <= 2^64 - 1 < (2^32 + v + 1) d
// (checked on the host for every d in [2^31, 2^32)): the 64-by-32 integer division
// above is a long software sequence on the GPU.  Kernel 2's division sites use it
// (C4 157.0 -> 154.6 ms); kernel 1 keeps the integer form (its C2 launch measured
// 0.6 % slower with this one).
DEV bool mg_recip_fits(uint32_t v, uint32_t d) {
    const uint64_t vd = (uint64_t)v * d;
    return (((uint64_t)d << 32) + vd) >= vd;          // no carry out of 2^64
}
DEV uint32_t mg_reciprocal_fp(uint32_t d) {
    double e = 18446744073709551616.0 / (double)d - 4294967296.0;
    e = e < 0.0 ? 0.0 : (e > 4294967295.0 ? 4294967295.0 : e);
    uint32_t v = (uint32_t)e;
    if (!mg_recip_fits(v, d)) v -= 1u;
    else if (v != 0xffffffffu && mg_recip_fits(v + 1u, d)) v += 1u;
    return v;
}
// (u1:u0) / d for u1 < d, d normalised, v = mg_reciprocal(d)  (MG 2011, Alg. 4)
DEV uint32_t mg_div21(uint32_t u1, uint32_t u0, uint32_t d, uint32_t v, uint32_t &rem) {
    const uint64_t p = (uint64_t)v * u1 + ((((uint64_t)u1 + 1u) << 32) | u0);
    uint32_t q1 = (uint32_t)(p >> 32);
    const uint32_t q0 = (uint32_t)p;
    uint32_t r = u0 - q1 * d;
    if (r > q0) { q1 -= 1u; r += d; }
    if (r >= d) { q1 += 1u; r -= d; }
    rem = r;
    return q1;
}

// SKIP (kernel 2): a quotient digit j is nonzero only when bitlen(a) - bitlen(b) >= 32 j (= dl),
// so a digit no lane of the wave needs is skipped with a wave-uniform branch (a zero digit
// leaves the remainder unchanged)
template <bool SKIP>
DEV void u_divmod_knuth(const U256 &a, const U256 &b, uint32_t lb, U256 &q, U256 &r, int dl) {
    const uint32_t s = 256u - lb;                       // normalisation shift, < 256
    const U256 vn = SKIP ? u_shl_n_w(b, s) : u_shl_n(b, s);
    const U256 lo = SKIP ? u_shl_n_w(a, s) : u_shl_n(a, s);
    U256 hi;
    if (SKIP && __ballot(s >= 32u) == 0ull) {
        // every lane's shift is below one limb: a's top s bits are all that move up
        hi = u_zero();
        hi.w[0] = s == 0u ? 0u : a.w[7] >> (32u - s);
    } else {
        hi = s == 0u ? u_zero() : (SKIP ? u_shr_n_w(a, 256u - s, 0u) : u_shr_n(a, 256u - s, 0u));
    }
    uint32_t u[17];
#pragma unroll
    for (int i = 0; i < 8; ++i) { u[i] = lo.w[i]; u[8 + i] = hi.w[i]; }
    u[16] = 0u;
    const uint32_t v7 = vn.w[7], v6 = vn.w[6];
    const uint32_t rcp = SKIP ? mg_reciprocal_fp(v7) : mg_reciprocal(v7);
    q = u_zero();
    // a < 2^256 so the digit at 2^256 is 0: u[15..8] < vn and the loop starts at 7
#pragma unroll
    for (int j = 7; j >= 0; --j) {
        if (SKIP && __ballot(dl >= 32 * j) == 0ull) continue;   // q.w[j] stays 0
        const uint32_t u2 = u[j + 8], u1 = u[j + 7], u0 = u[j + 6];
        uint32_t qh, rh;
        bool rh_ovf;
        if (u2 >= v7) {                                 // u2 == v7: qhat = 2^32 - 1
            qh = 0xffffffffu;
            const uint64_t t = (uint64_t)u1 + v7;       // rhat = u1 + v7
            rh = (uint32_t)t;
            rh_ovf = (t >> 32) != 0u;
        } else {
            qh = mg_div21(u2, u1, v7, rcp, rh);
            rh_ovf = false;
        }
        // refine: while qhat * v6 > (rhat : u0) decrement (at most twice)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (!rh_ovf) {
                const uint64_t lhs = (uint64_t)qh * v6;
                const uint64_t rhs = ((uint64_t)rh << 32) | u0;
                if (lhs > rhs) {
                    qh -= 1u;
                    const uint64_t t = (uint64_t)rh + v7;
                    rh = (uint32_t)t;
                    rh_ovf = (t >> 32) != 0u;
                }
            }
        }
        // u[j .. j+8] -= qh * vn
        uint32_t carry = 0u;
        unsigned borrow = 0u;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t p = (uint64_t)qh * vn.w[i] + carry;
            carry = (uint32_t)(p >> 32);
            u[j + i] = __builtin_subc(u[j + i], (uint32_t)p, borrow, &borrow);
        }
        unsigned neg = 0u;
        u[j + 8] = __builtin_subc(u[j + 8], carry, borrow, &neg);
        if (neg) {                                      // estimate one too large: add back
            qh -= 1u;
            unsigned c = 0u;
#pragma unroll
            for (int i = 0; i < 8; ++i) u[j + i] = __builtin_addc(u[j + i], vn.w[i], c, &c);
            u[j + 8] += c;
        }
        q.w[j] = qh;
    }
    U256 rn;
#pragma unroll
    for (int i = 0; i < 8; ++i) rn.w[i] = u[i];
    r = SKIP ? u_shr_n_w(rn, s, 0u) : u_shr_n(rn, s, 0u);
}

// KNUTH_ALL (kernel 2's division sites): Knuth D with zero digits skipped for every
// quotient length, instead of the shift-subtract loop below 32 quotient bits -- one
// estimated digit costs less than a few shift-subtract rounds (C4 190.96 -> 189.69 ms,
// profiles/r04/divab/).  Kernel 1 keeps the round-3 form.
template <bool KNUTH_ALL>
DEV void u_divmod_nz_t(const U256 &a, const U256 &b, U256 &q, U256 &r) {
    const uint32_t lb = u_bitlen(b), la = u_bitlen(a);
    if (u_popcount(b) == 1u) {
        const uint32_t k = lb - 1u;
        q = u_shr_n(a, k, 0u);
        r = u_and(a, u_sub(b, u_small(1)));
        return;
    }
    if (KNUTH_ALL ? __ballot(la >= lb) != 0ull : __ballot(la >= lb + 32u) != 0ull) {
        u_divmod_knuth<KNUTH_ALL>(a, b, lb, q, r, (int)la - (int)lb);   // some lane needs the long form
        return;
    }
    q = u_zero();
    r = a;
    if (la < lb) return;
    uint32_t d = la - lb;
    U256 bs = u_shl_n(b, d);
    for (uint32_t i = 0; i <= d; ++i) {
        const bool ge = !u_lt(r, bs);
        r = u_select(ge, u_sub(r, bs), r);
        // q = (q << 1) | ge
#pragma unroll
        for (int k = 7; k >= 1; --k) q.w[k] = (q.w[k] << 1) | (q.w[k - 1] >> 31);
        q.w[0] = (q.w[0] << 1) | (ge ? 1u : 0u);
        // bs >>= 1
#pragma unroll
        for (int k = 0; k < 7; ++k) bs.w[k] = (bs.w[k] >> 1) | (bs.w[k + 1] << 31);
        bs.w[7] >>= 1;
    }
}
DEV void u_divmod_nz(const U256 &a, const U256 &b, U256 &q, U256 &r) { u_divmod_nz_t<false>(a, b, q, r); }
DEV U256 z_udiv(const U256 &a, const U256 &b) {
    if (u_iszero(b)) return u_ones();
    U256 q, r;
    u_divmod_nz(a, b, q, r);
    return q;
}
DEV U256 z_urem(const U256 &a, const U256 &b) {
    if (u_iszero(b)) return a;
    U256 q, r;
    u_divmod_nz(a, b, q, r);
    return r;
}
DEV U256 z_sdiv(const U256 &a, const U256 &b) {
    const bool na = u_isneg(a), nb = u_isneg(b);
    if (u_iszero(b)) return na ? u_small(1) : u_ones();
    U256 q, r;
    u_divmod_nz(na ? u_neg(a) : a, nb ? u_neg(b) : b, q, r);
    return (na != nb) ? u_neg(q) : q;
}
DEV U256 z_srem(const U256 &a, const U256 &b) {
    if (u_iszero(b)) return a;
    const bool na = u_isneg(a), nb = u_isneg(b);
    U256 q, r;
    u_divmod_nz(na ? u_neg(a) : a, nb ? u_neg(b) : b, q, r);
    return na ? u_neg(r) : r;
}
// z3 bvsmod: remainder with the sign of the divisor
DEV U256 z_smod(const U256 &a, const U256 &b) {
    if (u_iszero(b)) return a;
    U256 r = z_srem(a, b);
    if (u_iszero(r) || u_isneg(r) == u_isneg(b)) return r;
    return u_add(r, b);
}
// pow(base, exp, 2^256), square-and-multiply over the exponent's bits
DEV U256 u_exp(U256 base, const U256 &e) {
    U256 acc = u_small(1);
    const uint32_t nb = u_bitlen(e);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        uint32_t word = e.w[k];
        for (uint32_t j = 0; j < 32u && 32u * k + j < nb; ++j) {
            if (word & 1u) acc = u_mul(acc, base);
            base = u_mul(base, base);
            word >>= 1;
        }
    }
    return acc;
}
