/*
 * u256_ref.h — 256-bit two's-complement arithmetic for the CPU oracle.
 *
 * TEST INFRASTRUCTURE ONLY: the oracle is the checker for the HIP kernels and
 * the CPU baseline of bench.py; the product path never links it.
 *
 * Deliberately a different representation from the device (4 x u64 limbs with
 * unsigned __int128 carries here, 8 x u32 limbs on the GPU) so that parity
 * between the two is evidence, not tautology.  Semantics are z3's bit-vector
 * semantics as used by mythril/laser/smt/bitvec.py:
 * division and remainder by zero are defined (bvudiv x 0 = 2^256-1,
 * bvurem x 0 = x, bvsdiv x 0 = x<0 ? 1 : 2^256-1, bvsrem x 0 = x).
 */
#ifndef U256_REF_H
#define U256_REF_H
#include <stdint.h>
#include <string.h>

typedef struct { uint64_t w[4]; } u256;  /* w[0] = least significant */
typedef unsigned __int128 u128;

static inline u256 u_zero(void) { u256 r = {{0, 0, 0, 0}}; return r; }
static inline u256 u_from64(uint64_t x) { u256 r = {{x, 0, 0, 0}}; return r; }
static inline int u_is_zero(u256 a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0; }
static inline int u_eq(u256 a, u256 b) {
    return a.w[0] == b.w[0] && a.w[1] == b.w[1] && a.w[2] == b.w[2] && a.w[3] == b.w[3];
}
static inline int u_lt(u256 a, u256 b) {
    for (int i = 3; i >= 0; --i)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i];
    return 0;
}
static inline int u_neg(u256 a) { return (int)(a.w[3] >> 63); }
static inline int u_slt(u256 a, u256 b) {
    int na = u_neg(a), nb = u_neg(b);
    if (na != nb) return na;
    return u_lt(a, b);
}
/* value fits in 64 bits */
static inline int u_fits64(u256 a) { return (a.w[1] | a.w[2] | a.w[3]) == 0; }

static inline u256 u_add(u256 a, u256 b) {
    u256 r; u128 c = 0;
    for (int i = 0; i < 4; ++i) { c += (u128)a.w[i] + b.w[i]; r.w[i] = (uint64_t)c; c >>= 64; }
    return r;
}
static inline u256 u_sub(u256 a, u256 b) {
    u256 r; uint64_t borrow = 0;
    for (int i = 0; i < 4; ++i) {
        uint64_t x = a.w[i], y = b.w[i];
        uint64_t d = x - y - borrow;
        borrow = (x < y) || (x == y && borrow) ? 1 : 0;
        r.w[i] = d;
    }
    return r;
}
static inline u256 u_mul(u256 a, u256 b) {
    uint64_t r[4] = {0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
        u128 c = 0;
        for (int j = 0; i + j < 4; ++j) {
            c += (u128)a.w[i] * b.w[j] + r[i + j];
            r[i + j] = (uint64_t)c; c >>= 64;
        }
    }
    u256 o; memcpy(o.w, r, sizeof r); return o;
}
static inline u256 u_and(u256 a, u256 b) { for (int i = 0; i < 4; ++i) a.w[i] &= b.w[i]; return a; }
static inline u256 u_or(u256 a, u256 b)  { for (int i = 0; i < 4; ++i) a.w[i] |= b.w[i]; return a; }
static inline u256 u_xor(u256 a, u256 b) { for (int i = 0; i < 4; ++i) a.w[i] ^= b.w[i]; return a; }
static inline u256 u_not(u256 a) { for (int i = 0; i < 4; ++i) a.w[i] = ~a.w[i]; return a; }
static inline u256 u_negate(u256 a) { return u_sub(u_zero(), a); }

static inline u256 u_shl(u256 a, u256 s) {
    if (!u_fits64(s) || s.w[0] >= 256) return u_zero();
    unsigned n = (unsigned)s.w[0], q = n / 64, r = n % 64;
    u256 o = u_zero();
    for (int i = 3; i >= (int)q; --i) {
        uint64_t v = a.w[i - q] << r;
        if (r && i - (int)q - 1 >= 0) v |= a.w[i - q - 1] >> (64 - r);
        o.w[i] = v;
    }
    return o;
}
static inline u256 u_lshr(u256 a, u256 s) {
    if (!u_fits64(s) || s.w[0] >= 256) return u_zero();
    unsigned n = (unsigned)s.w[0], q = n / 64, r = n % 64;
    u256 o = u_zero();
    for (int i = 0; i + (int)q < 4; ++i) {
        uint64_t v = a.w[i + q] >> r;
        if (r && i + (int)q + 1 < 4) v |= a.w[i + q + 1] << (64 - r);
        o.w[i] = v;
    }
    return o;
}
static inline u256 u_ashr(u256 a, u256 s) {
    int neg = u_neg(a);
    if (!u_fits64(s) || s.w[0] >= 256) {
        u256 o; uint64_t f = neg ? ~0ull : 0; for (int i = 0; i < 4; ++i) o.w[i] = f; return o;
    }
    u256 o = u_lshr(a, s);
    if (neg && s.w[0] > 0) {
        /* fill the top s bits with ones */
        u256 ones = u_not(u_zero());
        u256 keep = u_lshr(ones, s);
        o = u_or(o, u_not(keep));
    }
    return o;
}
static inline unsigned u_bitlen(u256 a) {
    for (int i = 3; i >= 0; --i)
        if (a.w[i]) return (unsigned)(64 * i + 64 - __builtin_clzll(a.w[i]));
    return 0;
}

/* Unsigned division, Knuth algorithm D on 64-bit digits with 128/64 steps.
 * b != 0 required. */
static void u_divmod_nz(u256 a, u256 b, u256 *q_out, u256 *r_out) {
    if (u_lt(a, b)) { if (q_out) *q_out = u_zero(); if (r_out) *r_out = a; return; }
    int n = 4; while (n > 0 && b.w[n - 1] == 0) --n;
    int m = 4; while (m > 0 && a.w[m - 1] == 0) --m;
    u256 q = u_zero();
    if (n == 1) {
        u128 rem = 0; uint64_t d = b.w[0];
        for (int i = m - 1; i >= 0; --i) {
            u128 cur = (rem << 64) | a.w[i];
            q.w[i] = (uint64_t)(cur / d); rem = cur % d;
        }
        if (q_out) *q_out = q;
        if (r_out) *r_out = u_from64((uint64_t)rem);
        return;
    }
    unsigned s = (unsigned)__builtin_clzll(b.w[n - 1]);
    uint64_t vn[4], un[5];
    for (int i = n - 1; i > 0; --i) vn[i] = (b.w[i] << s) | (s ? b.w[i - 1] >> (64 - s) : 0);
    vn[0] = b.w[0] << s;
    un[m] = s ? a.w[m - 1] >> (64 - s) : 0;
    for (int i = m - 1; i > 0; --i) un[i] = (a.w[i] << s) | (s ? a.w[i - 1] >> (64 - s) : 0);
    un[0] = a.w[0] << s;
    for (int j = m - n; j >= 0; --j) {
        u128 num = ((u128)un[j + n] << 64) | un[j + n - 1];
        u128 qhat = num / vn[n - 1];
        u128 rhat = num % vn[n - 1];
        while (qhat >> 64 || qhat * vn[n - 2] > ((rhat << 64) | un[j + n - 2])) {
            qhat -= 1; rhat += vn[n - 1];
            if (rhat >> 64) break;
        }
        /* multiply and subtract */
        u128 borrow = 0, carry = 0;
        for (int i = 0; i < n; ++i) {
            u128 p = qhat * vn[i] + carry;
            carry = p >> 64;
            u128 t = (u128)un[i + j] - (uint64_t)p - borrow;
            un[i + j] = (uint64_t)t;
            borrow = (t >> 64) ? 1 : 0;
        }
        u128 t = (u128)un[j + n] - (uint64_t)carry - borrow;
        un[j + n] = (uint64_t)t;
        if (t >> 64) { /* add back */
            qhat -= 1;
            u128 c = 0;
            for (int i = 0; i < n; ++i) {
                c += (u128)un[i + j] + vn[i];
                un[i + j] = (uint64_t)c; c >>= 64;
            }
            un[j + n] += (uint64_t)c;
        }
        q.w[j] = (uint64_t)qhat;
    }
    if (q_out) *q_out = q;
    if (r_out) {
        u256 r = u_zero();
        for (int i = 0; i < n; ++i)
            r.w[i] = (un[i] >> s) | (s && i + 1 <= n ? (un[i + 1] << (64 - s)) : 0);
        if (s == 0) for (int i = 0; i < n; ++i) r.w[i] = un[i];
        *r_out = r;
    }
}

/* z3 bvudiv / bvurem with their division-by-zero definitions */
static inline u256 z_udiv(u256 a, u256 b) {
    if (u_is_zero(b)) return u_not(u_zero());
    u256 q; u_divmod_nz(a, b, &q, 0); return q;
}
static inline u256 z_urem(u256 a, u256 b) {
    if (u_is_zero(b)) return a;
    u256 r; u_divmod_nz(a, b, 0, &r); return r;
}
static inline u256 z_sdiv(u256 a, u256 b) {
    int na = u_neg(a), nb = u_neg(b);
    if (u_is_zero(b)) return na ? u_from64(1) : u_not(u_zero());
    u256 ua = na ? u_negate(a) : a, ub = nb ? u_negate(b) : b;
    u256 q = z_udiv(ua, ub);
    return (na ^ nb) ? u_negate(q) : q;
}
static inline u256 z_srem(u256 a, u256 b) {
    if (u_is_zero(b)) return a;
    int na = u_neg(a), nb = u_neg(b);
    u256 ua = na ? u_negate(a) : a, ub = nb ? u_negate(b) : b;
    u256 r = z_urem(ua, ub);
    return na ? u_negate(r) : r;
}
/* z3 bvsmod: sign follows the divisor */
static inline u256 z_smod(u256 a, u256 b) {
    if (u_is_zero(b)) return a;
    u256 r = z_srem(a, b);
    if (u_is_zero(r)) return r;
    if (u_neg(r) != u_neg(b)) r = u_add(r, b);
    return r;
}

static inline u256 u_from_be(const uint8_t *p, size_t n) {  /* n <= 32 */
    u256 r = u_zero();
    for (size_t i = 0; i < n; ++i) {
        size_t bit = 8 * (n - 1 - i);
        r.w[bit / 64] |= (uint64_t)p[i] << (bit % 64);
    }
    return r;
}
static inline void u_to_be(u256 a, uint8_t out[32]) {
    for (int i = 0; i < 32; ++i) {
        int bit = 8 * (31 - i);
        out[i] = (uint8_t)(a.w[bit / 64] >> (bit % 64));
    }
}
static inline u256 u_from_limbs32(const uint32_t *l) {
    u256 r; for (int i = 0; i < 4; ++i) r.w[i] = (uint64_t)l[2 * i] | ((uint64_t)l[2 * i + 1] << 32);
    return r;
}
static inline void u_to_limbs32(u256 a, uint32_t *l) {
    for (int i = 0; i < 4; ++i) { l[2 * i] = (uint32_t)a.w[i]; l[2 * i + 1] = (uint32_t)(a.w[i] >> 32); }
}
#endif
