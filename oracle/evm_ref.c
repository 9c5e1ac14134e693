/*
 * evm_ref.c — CPU restatement of LASER's concrete instruction semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  Used by tests/ (parity checker), by
 * __graft_entry__.smoke() (checker) and by bench.py's cpu_baseline leg.  The
 * product path (mythril_amd/, libmythgpu.so) never links or calls it.
 *
 * It follows the reference line by line, quirks included:
 *   disassembly ............ mythril/disassembler/asm.py:99-148
 *   opcode table ........... mythril/support/opcodes.py:16-144
 *   jump resolution (>=) ... mythril/laser/ethereum/util.py:45-59
 *   step loop / halts ...... mythril/laser/ethereum/svm.py:293-337, 369-491
 *   gas accounting ......... instructions.py:143-176, machine_state.py:132-191
 *   opcode handlers ........ instructions.py:269-1959 (cited per case below)
 *   memory ................. state/memory.py:56-208
 *   storage (concrete K(0))  state/account.py:18-99
 *   calldata (concrete) .... state/calldata.py:121-165
 * The lane record layout is the host image declared in include/mythgpu.h; only
 * that data format is shared with the product — no code is.
 *
 * Semantics of a lane that stops: status/aux/steps/ret_* are written; pc, sp,
 * msize, gas_min/gas_max, stack, memory and storage keep their values from the
 * start of the instruction that stopped it (the pre-step state the reference
 * returns in final_states, svm.py:331-334).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "u256_ref.h"
#include "../include/mythgpu.h"

void orc_keccak256(const uint8_t *in, size_t len, uint8_t out[32]);

/* ----------------------------------------------------------- opcode table */
/* support/opcodes.py:16-144 — gas (min,max) and STACK[0] (items required by
 * the svm precheck, svm.py:391-402; with the table's own values: ADDMOD 2,
 * EXTCODESIZE 0, SSTORE 1, DUP/SWAP 0).  valid=0 => disassembles to INVALID. */
typedef struct { uint8_t valid; uint8_t req; uint32_t gmin, gmax; } orc_op;
static orc_op OPT[256];
static int opt_ready = 0;

static void set_op(int b, int req, uint32_t gmin, uint32_t gmax) {
    OPT[b].valid = 1; OPT[b].req = (uint8_t)req; OPT[b].gmin = gmin; OPT[b].gmax = gmax;
}
static void init_optable(void) {
    if (opt_ready) return;
    memset(OPT, 0, sizeof OPT);
    set_op(0x00, 0, 0, 0);                                  /* STOP */
    set_op(0x01, 2, 3, 3); set_op(0x02, 2, 5, 5); set_op(0x03, 2, 3, 3);
    set_op(0x04, 2, 5, 5); set_op(0x05, 2, 5, 5); set_op(0x06, 2, 5, 5);
    set_op(0x07, 2, 5, 5); set_op(0x08, 2, 8, 8); set_op(0x09, 3, 8, 8);
    set_op(0x0a, 2, 10, 340); set_op(0x0b, 2, 5, 5);
    for (int b = 0x10; b <= 0x14; ++b) set_op(b, 2, 3, 3);  /* LT GT SLT SGT EQ */
    set_op(0x15, 1, 3, 3);                                  /* ISZERO */
    set_op(0x16, 2, 3, 3); set_op(0x17, 2, 3, 3); set_op(0x18, 2, 3, 3);
    set_op(0x19, 1, 3, 3);                                  /* NOT */
    set_op(0x1a, 2, 3, 3); set_op(0x1b, 2, 3, 3); set_op(0x1c, 2, 3, 3); set_op(0x1d, 2, 3, 3);
    set_op(0x20, 2, 30, 30 + 6 * 8);                        /* SHA3 */
    set_op(0x30, 0, 2, 2); set_op(0x31, 1, 700, 700); set_op(0x32, 0, 2, 2);
    set_op(0x33, 0, 2, 2); set_op(0x34, 0, 2, 2); set_op(0x35, 1, 3, 3);
    set_op(0x36, 0, 2, 2); set_op(0x37, 3, 2, 2 + 3 * 768); set_op(0x38, 0, 2, 2);
    set_op(0x39, 3, 2, 2 + 3 * 768); set_op(0x3a, 0, 2, 2); set_op(0x3b, 0, 700, 700);
    set_op(0x3c, 4, 700, 700 + 3 * 768); set_op(0x3d, 0, 2, 2); set_op(0x3e, 3, 3, 3);
    set_op(0x3f, 1, 700, 700);
    set_op(0x40, 1, 20, 20);
    for (int b = 0x41; b <= 0x48; ++b) set_op(b, 0, 2, 2);
    set_op(0x50, 1, 2, 2); set_op(0x51, 1, 3, 96); set_op(0x52, 2, 3, 98);
    set_op(0x53, 2, 3, 98); set_op(0x54, 1, 800, 800); set_op(0x55, 1, 5000, 25000);
    set_op(0x56, 1, 8, 8); set_op(0x57, 2, 10, 10); set_op(0x58, 0, 2, 2);
    set_op(0x59, 0, 2, 2); set_op(0x5a, 0, 2, 2); set_op(0x5b, 0, 1, 1);
    set_op(0x5c, 0, 2, 2); set_op(0x5d, 0, 5, 5); set_op(0x5e, 1, 10, 10);
    for (int i = 1; i <= 32; ++i) set_op(0x5f + i, 0, 3, 3);   /* PUSH1..32 */
    for (int i = 1; i <= 16; ++i) { set_op(0x7f + i, 0, 3, 3); set_op(0x8f + i, 0, 3, 3); }
    for (int i = 0; i <= 4; ++i) set_op(0xa0 + i, i + 2, 375 * (i + 1), 375 * (i + 1) + 8 * 32);
    set_op(0xf0, 3, 32000, 32000); set_op(0xf5, 4, 32000, 32000);
    set_op(0xf1, 7, 700, 700 + 9000 + 25000); set_op(0xf2, 7, 700, 700 + 9000 + 25000);
    set_op(0xf3, 2, 0, 0); set_op(0xf4, 6, 700, 700 + 9000 + 25000);
    set_op(0xfa, 6, 700, 700 + 9000 + 25000); set_op(0xfd, 2, 0, 0);
    set_op(0xff, 1, 5000, 30000); set_op(0xfe, 0, 0, 0);
    opt_ready = 1;
}

int orc_opcode_info(uint32_t b, uint32_t *gmin, uint32_t *gmax, uint32_t *req) {
    init_optable();
    if (b > 255 || !OPT[b].valid) return -1;
    *gmin = OPT[b].gmin; *gmax = OPT[b].gmax; *req = OPT[b].req;
    return 0;
}

/* --------------------------------------------------------------- code */
typedef struct {
    uint8_t *bytes; size_t n_bytes;       /* full bytecode (CODECOPY/CODESIZE) */
    uint32_t n_instr;
    uint8_t *op;                          /* [n_instr] byte, 0xfe for INVALID  */
    uint32_t *addr;                       /* [n_instr] byte address            */
    u256 *push;                           /* [n_instr] push immediate          */
    uint8_t *argn;                        /* [n_instr] argument bytes present  */
    uint8_t *fent;                        /* [n_instr] function entry (0/1)    */
} orc_code;

#define ORC_MAX_CODES 4096
static orc_code CODES[ORC_MAX_CODES];
static int n_codes = 0;
/* optional coverage bytes per code (coverage_plugin.py:68-85 semantics of the
 * device's mg_coverage: an instruction is covered once a lane starts it) */
static uint8_t *COV[ORC_MAX_CODES];

/* Python's repr of a bytes object (the text `str(bytes)` returns), used by
 * asm.py:107-123 to look for "bzzr" in the last 43 bytes. */
static size_t py_bytes_repr(const uint8_t *p, size_t n, char *out) {
    int has_sq = 0, has_dq = 0;
    for (size_t i = 0; i < n; ++i) { has_sq |= p[i] == '\''; has_dq |= p[i] == '"'; }
    char q = (has_sq && !has_dq) ? '"' : '\'';
    size_t k = 0;
    out[k++] = 'b'; out[k++] = q;
    static const char HX[] = "0123456789abcdef";
    for (size_t i = 0; i < n; ++i) {
        uint8_t c = p[i];
        if (c == q || c == '\\') { out[k++] = '\\'; out[k++] = (char)c; }
        else if (c == '\t') { out[k++] = '\\'; out[k++] = 't'; }
        else if (c == '\n') { out[k++] = '\\'; out[k++] = 'n'; }
        else if (c == '\r') { out[k++] = '\\'; out[k++] = 'r'; }
        else if (c < 32 || c >= 127) {
            out[k++] = '\\'; out[k++] = 'x'; out[k++] = HX[c >> 4]; out[k++] = HX[c & 15];
        } else out[k++] = (char)c;
    }
    out[k++] = q; out[k] = 0;
    return k;
}

/* asm.py:99-148 */
static int disassemble(const uint8_t *bc, size_t len, orc_code *c) {
    size_t length = len;
    size_t tail = len < 43 ? len : 43;
    char rep[4 * 43 + 8];
    py_bytes_repr(bc + len - tail, tail, rep);
    if (strstr(rep, "bzzr")) length = len >= 43 ? len - 43 : 0;   /* length -= 43 */
    c->op = malloc(length + 1); c->addr = malloc(sizeof(uint32_t) * (length + 1));
    c->push = malloc(sizeof(u256) * (length + 1));
    c->argn = calloc(length + 1, 1);
    if (!c->op || !c->addr || !c->push || !c->argn) return -1;
    uint32_t k = 0;
    size_t a = 0;
    while (a < length) {
        uint8_t b = bc[a];
        c->addr[k] = (uint32_t)a;
        c->push[k] = u_zero();
        if (!OPT[b].valid) { c->op[k++] = 0xfe; a += 1; continue; }  /* INVALID */
        c->op[k] = b;
        if (b >= 0x60 && b <= 0x7f) {
            size_t np = (size_t)(b - 0x5f);
            /* argument = bytecode[a+1 : a+1+np] of the FULL bytecode; short
             * arguments are right-padded with zeros (instructions.py:316). */
            uint8_t buf[32]; memset(buf, 0, sizeof buf);
            for (size_t i = 0; i < np; ++i)
                if (a + 1 + i < len) buf[i] = bc[a + 1 + i];
            c->push[k] = u_from_be(buf, np);
            /* asm.py:137-139: the instruction's "argument" is the hex of the bytes
             * actually present (a PUSH at the end of the code is cut short) */
            c->argn[k] = (uint8_t)(a + 1 + np <= len ? np : len - (a + 1));
            a += np;
        }
        ++k; a += 1;
    }
    c->n_instr = k;
    c->bytes = malloc(len ? len : 1);
    if (!c->bytes) return -1;
    memcpy(c->bytes, bc, len);
    c->n_bytes = len;
    return 0;
}

/* int(instruction_list[k]["argument"], 16) as the reference parses it: the
 * hex text of the present argument bytes; -1 when it has none (the text "0x"
 * does not parse) or the value cannot be an instruction address. */
static int64_t argument_int(const orc_code *c, uint32_t k) {
    static const char HX[] = "0123456789abcdef";
    char txt[2 * 32 + 1];
    uint32_t m = 0;
    const uint32_t np = c->argn[k];
    if (np == 0) return -1;
    uint8_t be[32];
    u_to_be(c->push[k], be);                  /* the present bytes are the high ones */
    for (uint32_t j = 0; j < np; ++j) {
        const uint8_t v = be[32 - (uint32_t)(c->op[k] - 0x5f) + j];
        txt[m++] = HX[v >> 4]; txt[m++] = HX[v & 15];
    }
    txt[m] = 0;
    const char *p = txt;
    while (*p == '0' && p[1]) ++p;            /* int() ignores leading zeros */
    if (strlen(p) > 8) return -1;
    return (int64_t)strtoull(p, NULL, 16);
}

/* Disassembly.assign_bytecode (disassembly.py:36-56): the indices of
 * asm.find_op_code_sequence([("PUSH1".."PUSH4"), ("EQ",)]) (asm.py:66-94) give,
 * through get_function_info (disassembly.py:64-114), entry points = the argument
 * of instruction index + 2; address_to_function_name is keyed by them.  An
 * instruction is a function entry when its address is one (svm.py:617-631);
 * address 0 switches the name too ("fallback", :632-633). */
static int dispatcher_entries(orc_code *c) {
    c->fent = calloc(c->n_instr + 1, 1);
    if (!c->fent) return -1;
    if (c->n_instr) c->fent[0] = 1;
    for (uint32_t idx = 0; idx + 2 <= c->n_instr; ++idx) {
        const uint8_t o0 = c->op[idx], o1 = c->op[idx + 1];
        if (!(o0 >= 0x60 && o0 <= 0x63) || o1 != 0x14) continue;
        if (idx + 2 >= c->n_instr) continue;           /* IndexError: no entry point */
        const uint8_t o2 = c->op[idx + 2];
        if (!(o2 >= 0x60 && o2 <= 0x7f)) continue;     /* KeyError: no "argument" */
        const int64_t entry = argument_int(c, idx + 2);
        if (entry < 0) continue;
        for (uint32_t k = 0; k < c->n_instr; ++k)
            if ((int64_t)c->addr[k] == entry) { c->fent[k] = 1; break; }
    }
    return 0;
}

int orc_load_code(const uint8_t *bc, size_t len, uint32_t *code_id) {
    init_optable();
    if (n_codes >= ORC_MAX_CODES) return -1;
    orc_code *c = &CODES[n_codes];
    memset(c, 0, sizeof *c);
    if (disassemble(bc, len, c)) return -1;
    if (dispatcher_entries(c)) return -1;
    *code_id = (uint32_t)n_codes++;
    return 0;
}

/* The function-entry flags of a loaded code (n_instr bytes, 0/1). */
int orc_code_fentries(uint32_t id, uint8_t *out) {
    if (id >= (uint32_t)n_codes) return -1;
    memcpy(out, CODES[id].fent, CODES[id].n_instr);
    return 0;
}

void orc_reset_codes(void) {
    for (int i = 0; i < n_codes; ++i) {
        free(CODES[i].bytes); free(CODES[i].op); free(CODES[i].addr); free(CODES[i].push);
        free(CODES[i].argn); free(CODES[i].fent);
    }
    n_codes = 0;
    memset(COV, 0, sizeof COV);
}

/* Coverage sink of a loaded code (n_instr bytes owned by the caller; NULL = off). */
int orc_set_coverage(uint32_t id, uint8_t *bytes) {
    if (id >= (uint32_t)n_codes) return -1;
    COV[id] = bytes;
    return 0;
}

int orc_code_info(uint32_t id, uint32_t *n_instr, uint8_t *ops, uint32_t *addrs) {
    if (id >= (uint32_t)n_codes) return -1;
    *n_instr = CODES[id].n_instr;
    if (ops) memcpy(ops, CODES[id].op, CODES[id].n_instr);
    if (addrs) memcpy(addrs, CODES[id].addr, 4 * CODES[id].n_instr);
    return 0;
}

/* util.py:45-59: first instruction whose address >= target, else none (-1) */
static long resolve_jump(const orc_code *c, u256 target) {
    if (!u_fits64(target)) return -1;
    uint64_t t = target.w[0];
    /* addresses are increasing: binary search for the first addr >= t */
    uint32_t lo = 0, hi = c->n_instr;
    while (lo < hi) {
        uint32_t mid = (lo + hi) / 2;
        if ((uint64_t)c->addr[mid] >= t) hi = mid; else lo = mid + 1;
    }
    return lo < c->n_instr ? (long)lo : -1;
}

/* --------------------------------------------------------------- lanes */
typedef struct {
    uint64_t hook_mask[4];
    uint32_t max_steps;
    uint32_t max_depth;     /* 0 = unlimited */
    uint32_t horizon;       /* stop when the lane's cumulative steps reach it; 0 = none */
    uint32_t loop_bound;    /* BoundedLoopsStrategy bound; 0 = off */
} orc_params;

/* bounded_loops.py:49-113 restated literally: calculate_hash(i, j) is the OR of
 * trace[itr] << 8 (itr - i), kept here as a little-endian byte string so any
 * address width compares exactly (the device streams 16-bit addresses). */
static void seg_hash(const uint32_t *t, uint32_t a, uint32_t b, uint8_t *out, size_t cap) {
    memset(out, 0, cap);
    for (uint32_t itr = a; itr < b; ++itr)
        for (int k = 0; k < 4; ++k) out[(itr - a) + k] |= (uint8_t)(t[itr] >> (8 * k));
}

uint32_t orc_loop_count(const uint32_t *t, uint32_t n) {
    int64_t i;
    int found = 0;
    for (i = (int64_t)n - 3; i > 0; --i)
        if (t[i] == t[n - 2] && t[i + 1] == t[n - 1]) { found = 1; break; }
    if (!found) return 0;
    const uint32_t size = n - (uint32_t)i - 2;
    const size_t cap = (size_t)size + 4;
    uint8_t *key = (uint8_t *)malloc(cap), *cur = (uint8_t *)malloc(cap);
    seg_hash(t, (uint32_t)i + 1, n - 1, key, cap);
    uint32_t count = 1;
    for (int64_t j = i + 1; j >= 0; j -= size) {
        seg_hash(t, (uint32_t)j, (uint32_t)j + size, cur, cap);
        if (memcmp(cur, key, cap) != 0) break;
        count++;
    }
    free(key);
    free(cur);
    return count;
}

typedef struct {       /* working view of one lane */
    const mg_lane_soa *h;
    uint32_t i;
} lane_ref;

#define L32(f) (h->f[i])
static inline u256 stack_get(const mg_lane_soa *h, uint32_t i, uint32_t slot) {
    return u_from_limbs32(h->stack + ((size_t)i * h->stack_cap + slot) * 8);
}
static inline void stack_set(const mg_lane_soa *h, uint32_t i, uint32_t slot, u256 v) {
    u_to_limbs32(v, h->stack + ((size_t)i * h->stack_cap + slot) * 8);
}
static inline u256 env_get(const mg_lane_soa *h, uint32_t i, int w) {
    return u_from_limbs32(h->env + ((size_t)i * MG_ENV_WORDS + w) * 8);
}
static inline uint8_t *mem_of(const mg_lane_soa *h, uint32_t i) {
    return h->memory + (size_t)i * h->mem_cap;
}

#define BIG_END (1ull << 32)          /* start+size beyond this => certain OOG */
#define HUGE_GAS (1ull << 62)

/* ceil32(x) // 32 */
static inline uint64_t words_of(uint64_t x) { return (x + 31) / 32; }
static inline uint64_t mem_fee(uint64_t w) { return 3 * w + (w * w) / 512; }

/* Outcome of a memory extension request (machine_state.py:132-191). */
enum { MX_OK = 0, MX_OOG = 1, MX_ESCAPE = 2 };

/* mem_extend(start, size) on the working copies (msize, gmin, gmax).
 * Returns MX_OOG where the reference raises OutOfGasException inside
 * mem_extend (check_gas: min_gas_used > gas_limit=1e9), MX_ESCAPE where the
 * lane's page is too small (host takes over; nothing committed).
 * `later_min` >= 0: the instruction ends with an OOG check after adding
 * later_min (accumulate_gas, or RETURN's check_gas_usage_limit with 0); an
 * extension past the page that is certain to fail that check is reported as
 * the OOG it becomes instead of an escape. */
static int mem_extend(u256 start, u256 size, uint32_t *msize, uint64_t *gmin, uint64_t *gmax,
                      uint32_t mem_cap, long long later_min, uint64_t txlim) {
    u256 end = u_add(start, size);
    /* python ints: start + size does not wrap */
    int wrapped = u_lt(end, start);
    if (wrapped || !u_fits64(end) || end.w[0] > BIG_END) return MX_OOG;
    uint64_t e = end.w[0];
    if ((uint64_t)*msize > e) return MX_OK;          /* memory_size > start + size */
    uint64_t new_w = words_of(e), old_w = *msize / 32;
    if (new_w == old_w) return MX_OK;                /* m_extend == 0 */
    uint64_t fee = mem_fee(new_w) - mem_fee(old_w);
    uint64_t nmin = *gmin + fee;
    if (nmin > MG_MSTATE_GAS_LIMIT) return MX_OOG;
    if (new_w * 32 > mem_cap) {
        if (later_min >= 0 && (nmin + (uint64_t)later_min > MG_MSTATE_GAS_LIMIT ||
                               nmin + (uint64_t)later_min >= txlim))
            return MX_OOG;
        return MX_ESCAPE;
    }
    *gmin = nmin; *gmax += fee;
    *msize = (uint32_t)(new_w * 32);
    return MX_OK;
}

/* check_gas_usage_limit (instructions.py:143-160) after a gas add */
static inline int gas_oog(uint64_t gmin, uint64_t tx_limit) {
    return gmin > MG_MSTATE_GAS_LIMIT || gmin >= tx_limit;
}

static int storage_find(const mg_lane_soa *h, uint32_t i, u256 key) {
    uint32_t cnt = h->storage_count[i];
    const uint32_t *base = h->storage + (size_t)i * h->storage_cap * 16;
    for (uint32_t s = 0; s < cnt; ++s)
        if (u_eq(u_from_limbs32(base + s * 16), key)) return (int)s;
    return -1;
}

/* function-manager records: lane-major [n][rec_cap] words (include/mythgpu.h MG_REC_*) */
static uint32_t rec_put_word(const mg_lane_soa *h, uint32_t i, uint32_t at, u256 v) {
    uint32_t *q = h->rec + (size_t)i * h->rec_cap;
    for (int k = 0; k < 4; ++k) { q[at + 2 * k] = (uint32_t)v.w[k]; q[at + 2 * k + 1] = (uint32_t)(v.w[k] >> 32); }
    return at + 8;
}
/* step: the lane's steps count before this instruction (its BFS round) */
static uint32_t rec_put_head(const mg_lane_soa *h, uint32_t i, uint32_t at, uint32_t kind, uint32_t len, u256 r) {
    uint32_t *q = h->rec + (size_t)i * h->rec_cap;
    q[at] = kind; q[at + 1] = len; q[at + 2] = h->steps[i] - 1;
    return rec_put_word(h, i, at + 3, r);
}

static inline uint8_t mem_read_byte(const uint8_t *m, uint32_t msize, uint64_t k) {
    return k < msize ? m[k] : 0;
}

static int is_env_escape(uint8_t op) {
    switch (op) {
    case 0x31: /* BALANCE: symbolic balances array (instructions.py:906-931) */
    case 0x3b: case 0x3c: case 0x3f: /* EXTCODE*: world state / loader */
    case 0x40: case 0x41: case 0x42: case 0x43: case 0x44: /* BLOCKHASH..DIFFICULTY */
    case 0x46: case 0x47: case 0x48: /* CHAINID SELFBALANCE BASEFEE: symbolic */
    case 0x5a: /* GAS: new_bitvec("gas") */
    case 0x5d: case 0x5e: /* RETURNSUB JUMPSUB */
    case 0xf0: case 0xf1: case 0xf2: case 0xf4: case 0xf5: case 0xfa: /* CREATE/CALL* */
    case 0xff: /* SELFDESTRUCT */
        return 1;
    default:
        return 0;
    }
}

/* Run one lane to a stop or to max_steps.  Returns steps executed.
 *
 * Each handler runs in three phases so that a lane which stops keeps its
 * pre-step state exactly: (1) pops, checks, memory-extension gas and escapes
 * — no writes; (2) COMMIT_GAS(): accumulate_gas (instructions.py:162-176),
 * whose OOG is the only exception the reference raises after a mutator has
 * written; (3) writes.  The exception kind reported equals the reference's
 * because every other exception of a mutator precedes its writes. */
static uint32_t run_lane(const mg_lane_soa *h, uint32_t i, const orc_params *p) {
    const orc_code *c = &CODES[h->code_id[i]];
    uint32_t done = 0;
    uint8_t *mem = mem_of(h, i);
    for (;;) {
        if (h->status[i] != MG_RUNNING) break;
        if (p->max_depth && h->depth[i] >= p->max_depth) { h->status[i] = MG_DEPTH; break; }
        const uint32_t pc = h->pc[i];
        if (pc >= c->n_instr) { h->status[i] = MG_HALT_END; break; }
        const uint8_t op = c->op[pc];
        const uint32_t flags = h->flags[i];
        const int acked = (flags & MG_LANE_HOOK_ACK) && done == 0;
        const int hooked = ((p->hook_mask[op >> 6] >> (op & 63)) & 1) && !acked;
        const int budget = done >= p->max_steps || ((flags & MG_LANE_STEP1) && done >= 1) ||
                           (p->horizon && h->steps[i] >= p->horizon);
        /* BoundedLoopsStrategy.get_strategic_global_state (bounded_loops.py:115-145):
         * the state is popped -> its address joins the trace -> at a JUMPDEST the
         * loop count may drop it, before any hook runs.  A budget pause is not a
         * pop, and the re-fetch after a hook ACK is the same pop. */
        if (p->loop_bound && h->trace_cap && !acked && (hooked || !budget)) {
            uint32_t *tr = h->trace + (size_t)i * h->trace_cap;
            if (h->trace_len[i] >= h->trace_cap) {
                h->status[i] = MG_ESCAPE; h->aux[i] = op | (MG_ESC_TRACE << 8); break;
            }
            tr[h->trace_len[i]++] = c->addr[pc];
            if (op == 0x5b) {
                const uint32_t cnt = orc_loop_count(tr, h->trace_len[i]);
                const int creation = (flags & MG_LANE_CREATION) != 0;
                if (creation ? (cnt > p->loop_bound && cnt >= 128) : cnt > p->loop_bound) {
                    h->status[i] = MG_LOOP_BOUND; h->aux[i] = cnt; break;
                }
            }
        }
        if (hooked) { h->status[i] = MG_HOOK; h->aux[i] = op; break; }
        if (budget) break;
        if (is_env_escape(op) ||
            ((flags & MG_LANE_CREATION) && op >= 0x35 && op <= 0x38)) {
            /* creation lanes: CALLDATALOAD/SIZE/COPY and CODESIZE follow the
             * constructor-argument rules of instructions.py:887-1003 (CODECOPY
             * below: only offsets past the code read the symbolic calldata) */
            h->status[i] = MG_ESCAPE; h->aux[i] = op | (MG_ESC_OPCODE << 8); break;
        }

        const uint32_t sp0 = h->sp[i], msize0 = h->msize[i];
        uint32_t sp = sp0, msize = msize0, depth = h->depth[i];
        uint64_t gmin = h->gas_min[i], gmax = h->gas_max[i];
        const uint64_t txlim = h->gas_limit[i];
        uint32_t new_pc = pc + 1;
        int jumped = 0;           /* a JUMP / JUMPI successor (manage_cfg) */
        const orc_op *info = &OPT[op];
        int gas_by_table = 1, gas_done = 0;
        uint32_t status = MG_RUNNING, aux = 0;
        uint32_t rec_new = 0;   /* function-manager record log length after this step */

        done++; h->steps[i]++;
        if (COV[h->code_id[i]]) COV[h->code_id[i]][pc] = 1;

#define STOP_WITH(s, x) do { status = (s); aux = (x); goto stop; } while (0)
#define EXC(k) STOP_WITH(MG_VMEXC, (k))
#define ESC(r) do { h->steps[i]--; done--; STOP_WITH(MG_ESCAPE, op | ((r) << 8)); } while (0)
#define NEED_POP(k) do { if (sp < (uint32_t)(k)) EXC(MG_EXC_STACK_UNDERFLOW); } while (0)
#define POP() stack_get(h, i, --sp)
#define NEED_PUSH(k) do { if (sp + (k) > MG_STACK_LIMIT) EXC(MG_EXC_STACK_OVERFLOW); \
                          if (sp + (k) > h->stack_cap) ESC(MG_ESC_STACK); } while (0)
#define COMMIT_GAS() do { if (gas_by_table && !gas_done) { gmin += info->gmin; gmax += info->gmax; \
                          gas_done = 1; if (gas_oog(gmin, txlim)) EXC(MG_EXC_OUT_OF_GAS); } } while (0)
#define ZERO_FILL() do { if (msize > msize0) memset(mem + msize0, 0, msize - msize0); } while (0)
#define PUSH1(v) do { u256 v_ = (v); NEED_PUSH(1); COMMIT_GAS(); stack_set(h, i, sp++, v_); } while (0)
#define MEMX(st, sz, later) do { int mx_ = mem_extend((st), (sz), &msize, &gmin, &gmax, h->mem_cap, \
                                                      (later), txlim); \
                          if (mx_ == MX_OOG) EXC(MG_EXC_OUT_OF_GAS); \
                          if (mx_ == MX_ESCAPE) ESC(MG_ESC_MEMORY); } while (0)

        /* svm.py:391-402 stack precheck from the opcode table */
        if (sp < info->req) EXC(MG_EXC_STACK_UNDERFLOW);
        /* StateTransition write protection (instructions.py:188-193) */
        if ((flags & MG_LANE_STATIC) && (op == 0x55 || (op >= 0xa0 && op <= 0xa4)))
            EXC(MG_EXC_WRITE_PROTECTION);

        u256 a, b, cc, r;
        if (op >= 0x60 && op <= 0x7f) {                         /* PUSH (instructions.py:278-320) */
            PUSH1(c->push[pc]);
        } else if (op >= 0x80 && op <= 0x8f) {                  /* DUP (:322-331) */
            uint32_t k = op - 0x7f;
            NEED_POP(k);
            PUSH1(stack_get(h, i, sp - k));
        } else if (op >= 0x90 && op <= 0x9f) {                  /* SWAP (:333-343) */
            uint32_t k = op - 0x8f;
            NEED_POP(k + 1);
            a = stack_get(h, i, sp - 1); b = stack_get(h, i, sp - 1 - k);
            COMMIT_GAS();
            stack_set(h, i, sp - 1, b); stack_set(h, i, sp - 1 - k, a);
        } else if (op >= 0xa0 && op <= 0xa4) {                  /* LOG (:1710-1723): pops only */
            NEED_POP(2 + (op - 0xa0));
            sp -= 2 + (op - 0xa0);
        } else switch (op) {
        case 0x00: STOP_WITH(MG_HALT_STOP, 0);                   /* STOP (:1953-1959) */
        case 0x01: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_add(a, b)); break;
        case 0x02: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_mul(a, b)); break;
        case 0x03: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_sub(a, b)); break;
        /* DIV/SDIV/MOD/SMOD: 0 only when the divisor is provably 0 (:505-592) */
        case 0x04: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_is_zero(b) ? u_zero() : z_udiv(a, b)); break;
        case 0x05: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_is_zero(b) ? u_zero() : z_sdiv(a, b)); break;
        case 0x06: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_is_zero(b) ? u_zero() : z_urem(a, b)); break;
        case 0x07: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_is_zero(b) ? u_zero() : z_srem(a, b)); break;
        case 0x08: /* ADDMOD = URem(URem(a,n) + URem(b,n), n), 256-bit wrap (:594-607) */
            NEED_POP(3); a = POP(); b = POP(); cc = POP();
            PUSH1(z_urem(u_add(z_urem(a, cc), z_urem(b, cc)), cc)); break;
        case 0x09: /* MULMOD = URem(URem(a,n) * URem(b,n), n) (:609-622) */
            NEED_POP(3); a = POP(); b = POP(); cc = POP();
            PUSH1(z_urem(u_mul(z_urem(a, cc), z_urem(b, cc)), cc)); break;
        case 0x0a: { /* EXP concrete: pow(base, exp, 2**256) (exponent_function_manager.py:43-51) */
            NEED_POP(2); a = POP(); b = POP();
            if (h->rec_cap && h->rec_len[i] + MG_REC_HEADER + 16 > h->rec_cap) ESC(MG_ESC_RECORD);
            u256 acc = u_from64(1), base = a;
            unsigned nb = u_bitlen(b);
            for (unsigned bit = 0; bit < nb; ++bit) {
                if ((b.w[bit / 64] >> (bit % 64)) & 1) acc = u_mul(acc, base);
                base = u_mul(base, base);
            }
            if (h->rec_cap) {   /* the path gains acc == Power(a, b) */
                uint32_t at = rec_put_head(h, i, h->rec_len[i], MG_REC_EXP, 0, acc);
                at = rec_put_word(h, i, at, a);
                rec_new = rec_put_word(h, i, at, b);
            }
            PUSH1(acc); break;
        }
        case 0x0b: { /* SIGNEXTEND with the signed compare s0 <= 31 (:640-668) */
            NEED_POP(2); a = POP(); b = POP();
            u256 testbit = u_add(u_mul(a, u_from64(8)), u_from64(7));
            u256 set_tb = u_shl(u_from64(1), testbit);
            int sign_set = !u_is_zero(u_and(b, set_tb));
            int le31 = !u_slt(u_from64(31), a);       /* a <= 31, signed */
            if (le31) r = sign_set ? u_or(b, u_sub(u_zero(), set_tb))
                                   : u_and(b, u_sub(set_tb, u_from64(1)));
            else r = b;
            PUSH1(r); break;
        }
        case 0x10: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_from64(u_lt(a, b))); break;   /* ULT */
        case 0x11: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_from64(u_lt(b, a))); break;   /* UGT */
        case 0x12: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_from64(u_slt(a, b))); break;
        case 0x13: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_from64(u_slt(b, a))); break;
        case 0x14: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_from64(u_eq(a, b))); break;
        case 0x15: NEED_POP(1); a = POP(); PUSH1(u_from64(u_is_zero(a))); break;
        case 0x16: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_and(a, b)); break;
        case 0x17: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_or(a, b)); break;
        case 0x18: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_xor(a, b)); break;
        case 0x19: NEED_POP(1); a = POP(); PUSH1(u_not(a)); break;   /* TT256M1 - x */
        case 0x1a: { /* BYTE (:426-456) */
            NEED_POP(2); a = POP(); b = POP();
            if (!u_fits64(a) || a.w[0] > 31) r = u_zero();
            else r = u_and(u_lshr(b, u_from64((31 - a.w[0]) * 8)), u_from64(0xff));
            PUSH1(r); break;
        }
        case 0x1b: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_shl(b, a)); break;  /* value << shift */
        case 0x1c: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_lshr(b, a)); break;
        case 0x1d: NEED_POP(2); a = POP(); b = POP(); PUSH1(u_ashr(b, a)); break;
        case 0x20: { /* SHA3 (:1013-1051): its own gas, then mem_extend */
            gas_by_table = 0;
            NEED_POP(2); a = POP(); b = POP();
            uint64_t g = (!u_fits64(b) || b.w[0] > BIG_END) ? HUGE_GAS : 30 + 6 * words_of(b.w[0]);
            gmin += g; gmax += g;
            if (gas_oog(gmin, txlim)) EXC(MG_EXC_OUT_OF_GAS);
            MEMX(a, b, -1);
            uint64_t len = b.w[0];
            if (len && h->rec_cap && (uint64_t)h->rec_len[i] + MG_REC_HEADER + (len + 3) / 4 > h->rec_cap)
                ESC(MG_ESC_RECORD);
            uint8_t digest[32];
            if (len == 0) {
                /* keccak_function_manager.get_empty_keccak_hash (:87-93) */
                static const uint8_t EMPTY[32] = {
                    0xc5, 0xd2, 0x46, 0x01, 0x86, 0xf7, 0x23, 0x3c, 0x92, 0x7e, 0x7d,
                    0xb2, 0xdc, 0xc7, 0x03, 0xc0, 0xe5, 0x00, 0xb6, 0x53, 0xca, 0x82,
                    0x27, 0x3b, 0x7b, 0xfa, 0xd8, 0x04, 0x5d, 0x85, 0xa4, 0x70};
                memcpy(digest, EMPTY, 32);
            } else {
                uint64_t s0 = a.w[0];
                uint8_t *tmp = malloc(len);
                for (uint64_t k = 0; k < len; ++k) tmp[k] = mem_read_byte(mem, msize0, s0 + k);
                orc_keccak256(tmp, len, digest);
                if (h->rec_cap) {   /* keccak_function_manager.concrete_hashes[data] = hash */
                    uint32_t at = rec_put_head(h, i, h->rec_len[i], MG_REC_KECCAK, (uint32_t)len,
                                               u_from_be(digest, 32));
                    uint32_t *q = h->rec + (size_t)i * h->rec_cap;
                    for (uint64_t k = 0; k < len; k += 4) {
                        uint32_t w = 0;
                        for (uint64_t j = 0; j < 4; ++j)
                            w |= (uint32_t)(k + j < len ? tmp[k + j] : 0) << (24 - 8 * j);
                        q[at++] = w;
                    }
                    rec_new = at;
                }
                free(tmp);
            }
            NEED_PUSH(1);
            ZERO_FILL();
            stack_set(h, i, sp++, u_from_be(digest, 32));
            break;
        }
        case 0x30: PUSH1(env_get(h, i, MG_ENV_ADDRESS)); break;
        case 0x32: PUSH1(env_get(h, i, MG_ENV_ORIGIN)); break;
        case 0x33: PUSH1(env_get(h, i, MG_ENV_CALLER)); break;
        case 0x34: PUSH1(env_get(h, i, MG_ENV_CALLVALUE)); break;
        case 0x3a: PUSH1(env_get(h, i, MG_ENV_GASPRICE)); break;
        case 0x35: { /* CALLDATALOAD: byte (off+k) mod 2^256, 0 past the end (calldata.py:46-90,137-146) */
            NEED_POP(1); a = POP();
            uint8_t w[32];
            const uint8_t *cd = h->calldata + (size_t)i * h->calldata_cap;
            uint32_t cdl = h->calldata_len[i];
            for (int k = 0; k < 32; ++k) {
                u256 idx = u_add(a, u_from64((uint64_t)k));
                w[k] = (u_fits64(idx) && idx.w[0] < cdl) ? cd[idx.w[0]] : 0;
            }
            PUSH1(u_from_be(w, 32)); break;
        }
        case 0x36: PUSH1(u_from64(h->calldata_len[i])); break;
        case 0x37: { /* CALLDATACOPY (:806-891): nothing at all when size == 0 */
            NEED_POP(3); a = POP(); b = POP(); cc = POP();   /* mstart, dstart, size */
            if (!u_is_zero(cc)) {
                MEMX(a, cc, info->gmin);
                COMMIT_GAS();
                ZERO_FILL();
                const uint8_t *cd = h->calldata + (size_t)i * h->calldata_cap;
                uint32_t cdl = h->calldata_len[i];
                uint64_t n = cc.w[0], m0 = a.w[0];
                for (uint64_t k = 0; k < n; ++k) {
                    u256 idx = u_add(b, u_from64(k));
                    mem[m0 + k] = (u_fits64(idx) && idx.w[0] < cdl) ? cd[idx.w[0]] : 0;
                }
            }
            break;
        }
        case 0x38: PUSH1(u_from64(c->n_bytes)); break;   /* CODESIZE (:978-1003) */
        case 0x39: { /* CODECOPY -> _code_copy_helper (:1073-1250) */
            NEED_POP(3); a = POP(); b = POP(); cc = POP();   /* memory_offset, code_offset, size */
            /* creation tx with SymbolicCalldata: code_offset >= code_size copies
             * constructor arguments (instructions.py:1089-1098) -> host */
            if ((flags & MG_LANE_CREATION) && !(u_fits64(b) && b.w[0] < c->n_bytes)) ESC(MG_ESC_OPCODE);
            MEMX(a, cc, info->gmin);                        /* even for size 0 */
            COMMIT_GAS();
            ZERO_FILL();
            /* the copy stops at the end of the code: bytes past it are NOT written */
            uint64_t n = cc.w[0], m0 = a.w[0], ncopy = 0;
            if (u_fits64(b) && b.w[0] < c->n_bytes) {
                ncopy = c->n_bytes - b.w[0];
                if (ncopy > n) ncopy = n;
            }
            for (uint64_t k = 0; k < ncopy; ++k) mem[m0 + k] = c->bytes[b.w[0] + k];
            break;
        }
        case 0x3d:                                         /* RETURNDATASIZE: no last_return_data */
            if (flags & MG_LANE_RETDATA) ESC(MG_ESC_OPCODE);
            PUSH1(u_zero()); break;
        case 0x3e:                                         /* RETURNDATACOPY: last_return_data None */
            if (flags & MG_LANE_RETDATA) ESC(MG_ESC_OPCODE);
            NEED_POP(3); sp -= 3; break;
        case 0x45: PUSH1(u_from64(MG_MSTATE_GAS_LIMIT)); break;   /* GASLIMIT (:1427-1435) */
        case 0x50: NEED_POP(1); sp -= 1; break;
        case 0x51: { /* MLOAD (:1438-1451) */
            NEED_POP(1); a = POP();
            MEMX(a, u_from64(32), info->gmin);
            uint8_t w[32];
            for (int k = 0; k < 32; ++k) w[k] = mem_read_byte(mem, msize0, a.w[0] + k);
            COMMIT_GAS();
            ZERO_FILL();
            stack_set(h, i, sp++, u_from_be(w, 32));
            break;
        }
        case 0x52: { /* MSTORE (:1453-1470); mem_extend's OOG is swallowed, then accumulate_gas fails */
            NEED_POP(2); a = POP(); b = POP();
            MEMX(a, u_from64(32), info->gmin);
            COMMIT_GAS();
            ZERO_FILL();
            uint8_t w[32]; u_to_be(b, w);
            memcpy(mem + a.w[0], w, 32);
            break;
        }
        case 0x53: { /* MSTORE8 (:1472-1493) */
            NEED_POP(2); a = POP(); b = POP();
            MEMX(a, u_from64(1), info->gmin);
            COMMIT_GAS();
            ZERO_FILL();
            mem[a.w[0]] = (uint8_t)b.w[0];
            break;
        }
        case 0x54: { /* SLOAD over K(256,256,0) + stores (:1495-1506, account.py:43-74) */
            NEED_POP(1); a = POP();
            int s = storage_find(h, i, a);
            r = s < 0 ? u_zero()
                      : u_from_limbs32(h->storage + ((size_t)i * h->storage_cap + s) * 16 + 8);
            PUSH1(r); break;
        }
        case 0x55: { /* SSTORE (:1508-1518) */
            NEED_POP(2); a = POP(); b = POP();
            int s = storage_find(h, i, a);
            if (s < 0 && h->storage_count[i] >= h->storage_cap) ESC(MG_ESC_STORAGE);
            COMMIT_GAS();
            if (s < 0) {
                s = (int)h->storage_count[i]++;
                u_to_limbs32(a, h->storage + ((size_t)i * h->storage_cap + s) * 16);
            }
            u_to_limbs32(b, h->storage + ((size_t)i * h->storage_cap + s) * 16 + 8);
            break;
        }
        case 0x56: { /* JUMP (:1520-1556): gas 8 added by hand, no OOG check */
            gas_by_table = 0;
            NEED_POP(1); a = POP();
            long idx = resolve_jump(c, a);
            if (idx < 0 || c->op[idx] != 0x5b) EXC(MG_EXC_INVALID_JUMP);
            gmin += 8; gmax += 8; new_pc = (uint32_t)idx;
            jumped = 1;
            break;
        }
        case 0x57: { /* JUMPI (:1558-1636): gas 10 by hand, depth+1 on a taken side */
            gas_by_table = 0;
            NEED_POP(2); a = POP(); b = POP();   /* target, condition */
            if (u_is_zero(b)) {
                gmin += 10; gmax += 10; depth++; new_pc = pc + 1;
            } else {
                long idx = resolve_jump(c, a);
                if (idx < 0 || c->op[idx] != 0x5b) STOP_WITH(MG_HALT_DROPPED, 0);
                gmin += 10; gmax += 10; depth++; new_pc = (uint32_t)idx;
            }
            jumped = 1;
            break;
        }
        case 0x58: PUSH1(u_from64(c->addr[pc])); break;   /* PC (:1674-1687) */
        case 0x59: PUSH1(u_from64(msize)); break;          /* MSIZE */
        case 0x5b: break;                                   /* JUMPDEST */
        case 0x5c: EXC(MG_EXC_OUT_OF_GAS);                 /* BEGINSUB (:1638-1643) */
        case 0xf3: { /* RETURN (:1857-1874) */
            NEED_POP(2); a = POP(); b = POP();
            MEMX(a, b, 0);
            if (gas_oog(gmin, txlim)) EXC(MG_EXC_OUT_OF_GAS);
            h->ret_offset[i] = (uint32_t)a.w[0]; h->ret_len[i] = (uint32_t)b.w[0];
            STOP_WITH(MG_HALT_RETURN, 0);
        }
        case 0xfd: { /* REVERT (:1899-1934): no memory extension */
            NEED_POP(2); a = POP(); b = POP();
            h->ret_offset[i] = (uint32_t)a.w[0]; h->ret_len[i] = (uint32_t)b.w[0];
            STOP_WITH(MG_HALT_REVERT, 0);
        }
        case 0xfe: EXC(MG_EXC_INVALID_INSTRUCTION);        /* INVALID */
        default:
            /* unreachable: every valid byte is handled above or escaped */
            ESC(MG_ESC_OPCODE);
        }
        COMMIT_GAS();
        /* commit */
        h->pc[i] = new_pc; h->sp[i] = sp; h->msize[i] = msize; h->depth[i] = depth;
        h->gas_min[i] = gmin; h->gas_max[i] = gmax;
        if (rec_new) h->rec_len[i] = rec_new;
        /* manage_cfg -> _new_node_state (svm.py:549-637) on a JUMP / JUMPI successor */
        if (jumped && h->fent && new_pc < c->n_instr && c->fent[new_pc]) h->fent[i] = new_pc;
        continue;
    stop:
        h->status[i] = status; h->aux[i] = aux;
        break;
    }
    return done;
}

/* Step lanes [first, first+n) of a host image.  Returns the lane-steps. */
uint64_t orc_run_loop(const mg_lane_soa *h, uint32_t first, uint32_t n, const uint64_t hook_mask[4],
                      uint32_t max_steps, uint32_t max_depth, uint32_t horizon, uint32_t loop_bound) {
    init_optable();
    orc_params p;
    memcpy(p.hook_mask, hook_mask, sizeof p.hook_mask);
    p.max_steps = max_steps; p.max_depth = max_depth; p.horizon = horizon; p.loop_bound = loop_bound;
    uint64_t total = 0;
    for (uint32_t i = first; i < first + n; ++i) {
        if (h->code_id[i] >= (uint32_t)n_codes) { h->status[i] = MG_ESCAPE; continue; }
        const uint32_t done = run_lane(h, i, &p);
        /* HOOK_ACK covers one instruction: consumed once the lane has executed */
        if (done && (h->flags[i] & MG_LANE_HOOK_ACK)) h->flags[i] &= ~MG_LANE_HOOK_ACK;
        total += done;
    }
    return total;
}

uint64_t orc_run_until(const mg_lane_soa *h, uint32_t first, uint32_t n, const uint64_t hook_mask[4],
                       uint32_t max_steps, uint32_t max_depth, uint32_t horizon) {
    return orc_run_loop(h, first, n, hook_mask, max_steps, max_depth, horizon, 0);
}

uint64_t orc_run(const mg_lane_soa *h, uint32_t first, uint32_t n, const uint64_t hook_mask[4],
                 uint32_t max_steps, uint32_t max_depth) {
    return orc_run_until(h, first, n, hook_mask, max_steps, max_depth, 0);
}

/* Multi-threaded driver for the CPU baseline: one pthread per core over
 * disjoint lane ranges (lanes are independent paths). */
#include <pthread.h>
typedef struct { const mg_lane_soa *h; uint32_t first, n; const uint64_t *mask;
                 uint32_t max_steps, max_depth; uint64_t steps; } orc_job;
static void *orc_worker(void *arg) {
    orc_job *j = (orc_job *)arg;
    j->steps = orc_run(j->h, j->first, j->n, j->mask, j->max_steps, j->max_depth);
    return NULL;
}
uint64_t orc_run_mt(const mg_lane_soa *h, uint32_t first, uint32_t n, const uint64_t hook_mask[4],
                    uint32_t max_steps, uint32_t max_depth, uint32_t threads) {
    init_optable();
    if (threads <= 1 || n < threads) return orc_run(h, first, n, hook_mask, max_steps, max_depth);
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    orc_job jobs[256];
    uint32_t per = (n + threads - 1) / threads;
    uint32_t started = 0;
    for (uint32_t t = 0; t < threads; ++t) {
        uint32_t a = first + t * per;
        if (a >= first + n) break;
        uint32_t cnt = (a + per > first + n) ? first + n - a : per;
        jobs[t] = (orc_job){h, a, cnt, hook_mask, max_steps, max_depth, 0};
        pthread_create(&tid[t], NULL, orc_worker, &jobs[t]);
        started++;
    }
    uint64_t total = 0;
    for (uint32_t t = 0; t < started; ++t) { pthread_join(tid[t], NULL); total += jobs[t].steps; }
    return total;
}
