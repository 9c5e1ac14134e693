/*
 * bv_ref.c — CPU evaluator of kernel-2 constraint programs (TEST INFRASTRUCTURE ONLY).
 *
 * Restates, for the program format of mythril_amd/smt/program.py, what
 * ModelCache.check_quick_sat does per model (support_utils.py:60-68):
 * model.eval(And(constraints), model_completion=True), with z3 / SMT-LIB
 * bit-vector semantics (mythril/laser/smt/bitvec.py,
 * bitvec_helper.py, bool.py).  Variables absent from a model are 0 (model
 * completion).  Output per program: the first satisfying model index in
 * most-recently-used order (UINT32_MAX if none) and the satisfying count.
 *
 * Independent of the device code: 4 x u64 limbs (u256_ref.h) and its own
 * decoder; only the instruction format is shared.
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include "u256_ref.h"

enum {
    OP_COPY = 0, OP_ADD, OP_SUB, OP_MUL, OP_UDIV, OP_UREM, OP_SDIV, OP_SREM, OP_SMOD,
    OP_AND, OP_OR, OP_XOR, OP_NOT, OP_NEG, OP_SHL, OP_LSHR, OP_ASHR,
    OP_EQ, OP_ULT, OP_ULE, OP_UGT, OP_UGE, OP_SLT, OP_SLE, OP_SGT, OP_SGE,
    OP_BAND, OP_BOR, OP_BXOR, OP_BNOT, OP_BIMPLIES, OP_ITE, OP_EXTRACT, OP_CONCAT,
    OP_ZEXT, OP_SEXT, OP_ADD_NOOVF_U, OP_MUL_NOOVF_U, OP_SUB_NOUDF_U, OP_NE, OP_TAB,
    OP_UMIN, OP_UMAX, OP_SMIN, OP_SMAX, OP_RSUB, OP_RCONCAT
};

static u256 w_mask(u256 v, unsigned w) {
    if (w >= 256) return v;
    for (int i = 0; i < 4; ++i) {
        unsigned lo = 64u * i;
        if (w <= lo) v.w[i] = 0;
        else if (w < lo + 64) v.w[i] &= (w - lo == 64) ? ~0ull : ((1ull << (w - lo)) - 1);
    }
    return v;
}
static int w_bit(u256 v, unsigned b) { return (int)((v.w[b / 64] >> (b % 64)) & 1); }
static u256 w_sext(u256 v, unsigned w) {
    if (w == 0 || w >= 256 || !w_bit(v, w - 1)) return v;
    u256 ones = u_not(u_zero());
    return u_or(v, u_shl(ones, u_from64(w)));
}
static u256 w_bool(int b) { return u_from64(b ? 1 : 0); }

typedef struct {          /* model interpretations of arrays / functions */
    uint32_t n_tables;
    const uint32_t *start, *count, *entries, *dflt;
} tables_t;

typedef struct {
    const uint32_t *insns, *prog_off, *consts, *values;
    uint32_t n_vars, n_models, n_slots;
    uint32_t *first_sat, *sat_count;
    uint32_t d0, d1;
    uint64_t *bits;          /* optional [n_dags][ceil(n_models / 64)]: model m satisfies DAG d */
    const tables_t *tab;
} job_t;

/* Value of table `imm` (index | part << 20 | lo << 21) at key (k0, k1) in model m:
 * the listed entry with that key, else the default; bits [256 part + lo, ...). */
static u256 table_lookup(const job_t *j, u256 k0, u256 k1, uint32_t imm, uint32_t m) {
    const uint32_t t = imm & 0xfffffu, part = (imm >> 20) & 1u, lo = (imm >> 21) & 0xffu;
    const size_t tm = (size_t)t * j->n_models + m;
    u256 v = u_from_limbs32(j->tab->dflt + tm * 16 + part * 8);
    for (uint32_t k = 0; k < j->tab->count[tm]; ++k) {
        const uint32_t *e = j->tab->entries + ((size_t)j->tab->start[tm] + k) * 32;
        if (u_eq(u_from_limbs32(e), k0) && u_eq(u_from_limbs32(e + 8), k1)) {
            v = u_from_limbs32(e + 16 + part * 8);
            break;
        }
    }
    return u_lshr(v, u_from64(lo));
}

static u256 fetch(const job_t *j, u256 acc, const u256 *slots, uint32_t ref, uint32_t m) {
    uint32_t kind = ref >> 30, idx = ref & 0x3fffffffu;
    switch (kind) {
    case 0: return acc;
    case 1: return slots[idx];
    case 2: return u_from_limbs32(j->values + ((size_t)idx * j->n_models + m) * 8);
    default: return u_from_limbs32(j->consts + (size_t)idx * 8);
    }
}

static int eval_one(const job_t *j, uint32_t d, uint32_t m) {
    u256 slots[16];
    memset(slots, 0, sizeof slots);
    u256 acc = u_zero();
    for (uint32_t p = j->prog_off[d]; p < j->prog_off[d + 1]; ++p) {
        const uint32_t *w = j->insns + 4 * (size_t)p;
        uint32_t op = w[0] & 0xff, width = (w[0] >> 8) & 0x1ff;
        u256 a = fetch(j, acc, slots, w[1], m), r;
        u256 b = u_zero(), c = u_zero();
        int unary = op == OP_COPY || op == OP_NOT || op == OP_NEG || op == OP_BNOT ||
                    op == OP_EXTRACT || op == OP_ZEXT || op == OP_SEXT;
        if (!unary) b = fetch(j, acc, slots, w[2], m);
        if (op == OP_ITE) c = fetch(j, acc, slots, w[3], m);
        unsigned ow = w[3];  /* operand width for compares / concat low width */
        switch (op) {
        case OP_COPY: case OP_ZEXT: r = a; break;
        case OP_ADD: r = u_add(a, b); break;
        case OP_SUB: r = u_sub(a, b); break;
        case OP_MUL: r = u_mul(a, b); break;
        case OP_UDIV: r = u_is_zero(b) ? w_mask(u_not(u_zero()), width) : z_udiv(a, b); break;
        case OP_UREM: r = z_urem(a, b); break;
        case OP_SDIV: r = z_sdiv(w_sext(a, width), w_sext(b, width)); break;
        case OP_SREM: r = z_srem(w_sext(a, width), w_sext(b, width)); break;
        case OP_SMOD: r = z_smod(w_sext(a, width), w_sext(b, width)); break;
        case OP_AND: r = u_and(a, b); break;
        case OP_OR: r = u_or(a, b); break;
        case OP_XOR: r = u_xor(a, b); break;
        case OP_NOT: r = u_not(a); break;
        case OP_NEG: r = u_negate(a); break;
        case OP_SHL: r = (u_fits64(b) && b.w[0] < width) ? u_shl(a, b) : u_zero(); break;
        case OP_LSHR: r = (u_fits64(b) && b.w[0] < width) ? u_lshr(a, b) : u_zero(); break;
        case OP_ASHR: {
            u256 sa = w_sext(a, width);
            r = (u_fits64(b) && b.w[0] < width) ? u_ashr(sa, b) : u_ashr(sa, u_from64(255));
            break;
        }
        case OP_EQ: r = w_bool(u_eq(a, b)); break;
        case OP_NE: r = w_bool(!u_eq(a, b)); break;
        case OP_ULT: r = w_bool(u_lt(a, b)); break;
        case OP_ULE: r = w_bool(!u_lt(b, a)); break;
        case OP_UGT: r = w_bool(u_lt(b, a)); break;
        case OP_UGE: r = w_bool(!u_lt(a, b)); break;
        case OP_SLT: r = w_bool(u_slt(w_sext(a, ow), w_sext(b, ow))); break;
        case OP_SLE: r = w_bool(!u_slt(w_sext(b, ow), w_sext(a, ow))); break;
        case OP_SGT: r = w_bool(u_slt(w_sext(b, ow), w_sext(a, ow))); break;
        case OP_SGE: r = w_bool(!u_slt(w_sext(a, ow), w_sext(b, ow))); break;
        case OP_BAND: r = w_bool((a.w[0] & b.w[0]) & 1); break;
        case OP_BOR: r = w_bool((a.w[0] | b.w[0]) & 1); break;
        case OP_BXOR: r = w_bool((a.w[0] ^ b.w[0]) & 1); break;
        case OP_BNOT: r = w_bool(!(a.w[0] & 1)); break;
        case OP_BIMPLIES: r = w_bool(!(a.w[0] & 1) || (b.w[0] & 1)); break;
        case OP_ITE: r = (a.w[0] & 1) ? b : c; break;
        case OP_EXTRACT: r = u_lshr(a, u_from64(w[2] & 0xff)); break;
        case OP_CONCAT: r = u_or(u_shl(a, u_from64(ow)), b); break;
        case OP_SEXT: r = w_sext(a, w[2]); break;
        case OP_ADD_NOOVF_U: {
            /* z3 bvadd_noovfl (unsigned): the (w+1)-bit sum has a zero top bit */
            u256 s = u_add(a, b);
            int ovf = ow >= 256 ? u_lt(s, a) : !u_is_zero(u_lshr(s, u_from64(ow)));
            r = w_bool(!ovf);
            break;
        }
        case OP_MUL_NOOVF_U: {
            /* z3 bvumul_noovfl: the high w bits of the 2w-bit product are zero.
             * Computed exactly with a 512-bit product. */
            uint64_t prod[8] = {0};
            for (int i2 = 0; i2 < 4; ++i2) {
                u128 carry = 0;
                for (int k = 0; k < 4; ++k) {
                    u128 t = (u128)a.w[i2] * b.w[k] + prod[i2 + k] + carry;
                    prod[i2 + k] = (uint64_t)t; carry = t >> 64;
                }
                prod[i2 + 4] = (uint64_t)carry;
            }
            int ovf = 0;
            for (unsigned bit = ow; bit < 512; ++bit)
                if ((prod[bit / 64] >> (bit % 64)) & 1) { ovf = 1; break; }
            r = w_bool(!ovf);
            break;
        }
        case OP_SUB_NOUDF_U: r = w_bool(!u_lt(a, b)); break;
        case OP_TAB: r = table_lookup(j, a, b, w[3], m); break;
        case OP_UMIN: r = u_lt(b, a) ? b : a; break;
        case OP_UMAX: r = u_lt(a, b) ? b : a; break;
        case OP_SMIN: r = u_slt(w_sext(b, width), w_sext(a, width)) ? b : a; break;
        case OP_SMAX: r = u_slt(w_sext(a, width), w_sext(b, width)) ? b : a; break;
        case OP_RSUB: r = u_sub(b, a); break;
        case OP_RCONCAT: r = u_or(u_shl(b, u_from64(ow)), a); break;   /* a low (ow bits), b high */
        default: r = u_zero(); break;
        }
        r = w_mask(r, width);
        acc = r;
        if ((w[0] >> 17) & 1) slots[(w[0] >> 18) & 0xf] = r;
    }
    return (int)(acc.w[0] & 1);
}

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (uint32_t d = j->d0; d < j->d1; ++d) {
        uint32_t first = 0xffffffffu, cnt = 0;
        const uint32_t words = (j->n_models + 63u) / 64u;
        for (uint32_t m = 0; m < j->n_models; ++m)
            if (eval_one(j, d, m)) {
                if (first == 0xffffffffu) first = m;
                ++cnt;
                if (j->bits) j->bits[(size_t)d * words + m / 64u] |= 1ull << (m % 64u);
            }
        j->first_sat[d] = first;
        if (j->sat_count) j->sat_count[d] = cnt;
    }
    return NULL;
}

/* Evaluate programs [d_first, d_first+d_count) on every model; with `bits`
 * (zeroed by the caller) also the per-model satisfaction bitmap (mg_eval_bits). */
void orb_eval_tab_bits(const uint32_t *insns, const uint32_t *prog_off, const uint32_t *consts,
                       const uint32_t *values, uint32_t n_vars, uint32_t n_models, uint32_t n_slots,
                       uint32_t d_first, uint32_t d_count, uint32_t *first_sat, uint32_t *sat_count,
                       uint32_t threads, uint32_t n_tables, const uint32_t *tab_start,
                       const uint32_t *tab_count, const uint32_t *tab_entries, const uint32_t *tab_default,
                       uint64_t *bits);

void orb_eval_tab(const uint32_t *insns, const uint32_t *prog_off, const uint32_t *consts,
                  const uint32_t *values, uint32_t n_vars, uint32_t n_models, uint32_t n_slots,
                  uint32_t d_first, uint32_t d_count, uint32_t *first_sat, uint32_t *sat_count,
                  uint32_t threads, uint32_t n_tables, const uint32_t *tab_start,
                  const uint32_t *tab_count, const uint32_t *tab_entries, const uint32_t *tab_default) {
    orb_eval_tab_bits(insns, prog_off, consts, values, n_vars, n_models, n_slots, d_first, d_count,
                      first_sat, sat_count, threads, n_tables, tab_start, tab_count, tab_entries, tab_default,
                      NULL);
}

void orb_eval_tab_bits(const uint32_t *insns, const uint32_t *prog_off, const uint32_t *consts,
                       const uint32_t *values, uint32_t n_vars, uint32_t n_models, uint32_t n_slots,
                       uint32_t d_first, uint32_t d_count, uint32_t *first_sat, uint32_t *sat_count,
                       uint32_t threads, uint32_t n_tables, const uint32_t *tab_start,
                       const uint32_t *tab_count, const uint32_t *tab_entries, const uint32_t *tab_default,
                       uint64_t *bits) {
    const tables_t tab = {n_tables, tab_start, tab_count, tab_entries, tab_default};
    if (threads < 1) threads = 1;
    if (threads > 128) threads = 128;
    if (threads > d_count) threads = d_count ? d_count : 1;
    job_t jobs[128];
    pthread_t tid[128];
    uint32_t per = (d_count + threads - 1) / threads;
    uint32_t started = 0;
    for (uint32_t t = 0; t < threads; ++t) {
        uint32_t a = d_first + t * per;
        if (a >= d_first + d_count) break;
        uint32_t b = a + per > d_first + d_count ? d_first + d_count : a + per;
        jobs[t] = (job_t){insns, prog_off, consts, values, n_vars, n_models, n_slots,
                          first_sat, sat_count, a, b, bits, &tab};
        if (threads == 1) worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, worker, &jobs[t]);
        started++;
    }
    if (threads > 1)
        for (uint32_t t = 0; t < started; ++t) pthread_join(tid[t], NULL);
}

void orb_eval(const uint32_t *insns, const uint32_t *prog_off, const uint32_t *consts,
              const uint32_t *values, uint32_t n_vars, uint32_t n_models, uint32_t n_slots,
              uint32_t d_first, uint32_t d_count, uint32_t *first_sat, uint32_t *sat_count,
              uint32_t threads) {
    orb_eval_tab(insns, prog_off, consts, values, n_vars, n_models, n_slots, d_first, d_count,
                 first_sat, sat_count, threads, 0, NULL, NULL, NULL, NULL);
}
