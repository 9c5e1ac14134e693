// sym_step.cuh — symbolic lanes: the expression arena.
//
// A lane flagged LANE_SYMBOLIC carries symbolic stack words: every stack slot has
// a tag (0 = concrete value in the stack row, else 1 + the index of the arena
// node that defines it).  Sources are symbolic calldata (CALLDATALOAD /
// CALLDATASIZE of a SymbolicCalldata, state/calldata.py:214-262) and symbolic
// environment words (sender, origin, call value, gas price of a symbolic
// transaction, transaction/symbolic.py:105-150); the ALU opcodes build nodes
// over them (instructions.py:356-760), and a JUMPI on a symbolic condition stops
// the lane with MG_FORK so the host forks it with the two branch conditions
// (instructions.py:1558-1636) and checks them with kernel 2.  Everything the
// device has no symbolic semantics for (a symbolic memory offset or value,
// storage key or value, jump target, SHA3 input, EXP ...) stops the lane with
// MG_ESC_SYMBOLIC before the instruction: the host's escape handler (the
// reference's own execute_state) runs it.  Concrete instructions of a symbolic
// lane run through the concrete general handler (slow_step), so their
// semantics are kernel 1's, bit for bit.
//
// One thread per lane, stack rows in HBM (no LDS window): symbolic lanes are the
// minority of a batch (the concrete ones run in k_lane_step, which skips these).
//
// Taint lanes (MG_LANE_TAINT) run here too: every stack slot
// carries an object handle and every object an annotation mask over the lane's
// atoms (include/mythgpu.h "taint lanes"), so the reference's annotation sets
// follow the words exactly as laser/smt/expression.py and bitvec.py move them --
// unions through the ALU, one shared object per DUP and per environment word,
// nothing through concrete memory or storage -- and the batch-safe hooks of
// mythril_amd/laser/taint.py run here as per-opcode actions instead of a host
// round trip.
#pragma once

#define ST_FORK 11u
#define ESC_SYMBOLIC 7u
#define ESC_ARENA 8u
#define LANE_SYMBOLIC 16u
#define LANE_SYMCD 32u
#define LANE_SYMENV_SHIFT 6u
#define SYM_CDLOAD 1u
#define SYM_CDSIZE 2u
#define SYM_ENV 3u
#define SYM_BIN 4u
#define SYM_UN 5u
#define SYM_CONST 0x80000000u

DEV uint32_t sym_tag(const DevSym &S, size_t N, uint32_t lane, uint32_t slot) {
    return S.stag[(size_t)slot * N + lane];
}
DEV void sym_set_tag(const DevSym &S, size_t N, uint32_t lane, uint32_t slot, uint32_t t) {
    S.stag[(size_t)slot * N + lane] = t;
}
DEV uint32_t sym_width(const DevSym &S, size_t N, uint32_t lane, uint32_t tag) {
    return tag ? (S.node[(size_t)(tag - 1u) * N + lane].x >> 8) : 256u;
}
// operand reference of a stack word: its node, or a new constant-table entry
DEV bool sym_ref(const DevSym &S, size_t N, uint32_t lane, uint32_t tag, const U256 &v, uint32_t &nc,
                 uint32_t &ref) {
    if (tag) { ref = tag - 1u; return true; }
    if (nc >= S.const_cap) return false;
    st_word(gv(S.cval), (size_t)nc * N + lane, v);
    ref = SYM_CONST | nc;
    ++nc;
    return true;
}

DEV bool sym_node_push(const DevSym &S, size_t N, uint32_t lane, uint32_t kind_width, uint32_t y, uint32_t z,
                       uint32_t w, uint32_t &nn, uint32_t &tag) {
    if (nn >= S.node_cap) return false;
    S.node[(size_t)nn * N + lane] = make_uint4(kind_width, y, z, w);
    tag = nn + 1u;
    ++nn;
    return true;
}

// ---- symbolic memory, storage and SHA3 (ABI v7) ----------------------------------
#define LANE_SYMSTORE 4096u
#define LANE_MEMTAG 8192u
#define LANE_SYMBAL 32768u
#define LANE_SYMRDS 65536u
#define LANE_BALANCE 131072u
#define LANE_SYMBLOCK 262144u
#define SYM_SLOAD 6u
#define SYM_KECCAK 7u
#define SYM_EXTRACT 8u
#define SYM_CONCAT 9u
#define SYM_TERM 10u
#define SYM_NONE 0xffffffffu
#define SYM_CDBYTE 12u
#define SYM_CDBYTEX 13u
#define SYM_MSTOREK 14u
#define SYM_MLOADK 15u
#define SYM_BALANCE 16u
// A tagged word the host can only decode to a symbolic term: a fresh calldata word
// or size, an environment word, a keccak of symbolic data.  Any other node (an
// ALU result such as x - x, an MLOADK of a word stored concretely, a BALANCE of a
// known account, a store-chain read) may decode to a constant after simplify, and
// then the reference takes a concrete branch (util.get_concrete_int) -- the device
// leaves those to the host.
DEV bool sym_never_const(const DevSym &S, size_t N, uint32_t lane, uint32_t tag) {
    if (!tag) return false;
    const uint32_t kind = S.node[(size_t)(tag - 1u) * N + lane].x & 0xffu;
    return kind == SYM_CDLOAD || kind == SYM_CDSIZE || kind == SYM_ENV || kind == SYM_KECCAK;
}

DEV uint32_t mtag_at(const DevSym &S, size_t N, uint32_t lane, uint32_t off) { return S.mtag[(size_t)off * N + lane]; }
DEV void set_mtag(const DevSym &S, size_t N, uint32_t lane, uint32_t off, uint32_t t) {
    S.mtag[(size_t)off * N + lane] = t;
}
// any symbolic byte in memory [off, off + len) (bytes past msize are zero)
DEV bool mtag_any(const DevSym &S, size_t N, uint32_t lane, uint32_t off, uint32_t len, uint32_t msize) {
    const uint32_t end = min(off + len, msize);
    for (uint32_t p = off; p < end; ++p)
        if (mtag_at(S, N, lane, p)) return true;
    return false;
}

// Whether operand refs x and y denote the same term.  z3 terms are hash-consed,
// so the Select-over-Store rewrites of simplify (storage reads, account.py:75)
// compare indices by identity; here: equal refs, equal constants, or nodes with
// equal headers whose operands are the same terms, walked with an explicit
// stack.  A comparison deeper than the stack answers false, so the device keeps
// a Select node the host's decode then folds (decoding decides the term).
// The planes come as pointers, not the kernel's DevSym: a reference argument
// to a call forces the kernel's by-value argument structs into per-lane scratch
// for the whole launch (every lane wrote them at entry: ~330 bytes a lane).
__device__ __noinline__ bool sym_same(const uint4 *node, const uint4 *cval, size_t N, uint32_t lane, uint32_t x,
                                      uint32_t y) {
    uint32_t st[32];
    int top = 0;
    st[top++] = x;
    st[top++] = y;
    while (top) {
        const uint32_t b = st[--top], a = st[--top];
        if (a == b) continue;
        const bool ca = (a & SYM_CONST) != 0u, cb = (b & SYM_CONST) != 0u;
        if (ca || cb) {
            if (!(ca && cb)) return false;
            if (!u_eq(ld_word(gv(cval), (size_t)(a & ~SYM_CONST) * N + lane),
                      ld_word(gv(cval), (size_t)(b & ~SYM_CONST) * N + lane)))
                return false;
            continue;
        }
        const uint4 na = node[(size_t)a * N + lane], nb = node[(size_t)b * N + lane];
        if (na.x != nb.x || na.w != nb.w) return false;
        const uint32_t kind = na.x & 0xffu;
        const bool yref = kind != SYM_CDSIZE && kind != SYM_ENV && kind != SYM_TERM;
        const bool zref = kind == SYM_BIN || kind == SYM_CONCAT;
        if (!yref && na.y != nb.y) return false;
        if (!zref && na.z != nb.z) return false;      // SLOAD: the chain length
        if (top + 4 > 32) return false;
        if (yref) { st[top++] = na.y; st[top++] = nb.y; }
        if (zref) { st[top++] = na.z; st[top++] = nb.z; }
    }
    return true;
}

// Memory [off, off + len) as one operand, the parts of simplify(Concat(bytes))
// (memory.py:56-82, instructions.py:1032-1039): constant runs (<= 32 bytes each),
// runs of consecutive bytes of one node's word (an EXTRACT node, or the node
// itself for its 32 bytes in order), joined left to right by CONCAT nodes.  The
// host's decode joins the parts the same way expr.simplify_concat joins bytes.
// False when the arena or the constant table is full.
// S by value (a few registers) and the memory plane as a pointer: see sym_same.
__device__ __noinline__ bool sym_mem_ref(const DevSym S, const uint32_t *mem, size_t N, uint32_t lane,
                                         uint32_t off, uint32_t len, uint32_t msize, uint32_t &nn, uint32_t &nc,
                                         uint32_t &ref) {
    uint32_t acc = SYM_NONE, accw = 0u, k = 0u;
    while (k < len) {
        const uint32_t p = off + k;
        const uint32_t tag = p < msize ? mtag_at(S, N, lane, p) : 0u;
        uint32_t part, pw;
        if (tag == 0u) {
            U256 v = u_zero();
            uint32_t run = 0u;
            while (k < len && run < 32u) {
                const uint32_t q = off + k;
                if (q < msize && mtag_at(S, N, lane, q) != 0u) break;
                v = u_shl_n(v, 8u);
                v.w[0] |= q < msize ? (gp(mem)[(size_t)(q >> 2) * N + lane] >> (24u - 8u * (q & 3u))) & 0xffu
                                    : 0u;
                ++run;
                ++k;
            }
            if (nc >= S.const_cap) return false;
            st_word(gv(S.cval), (size_t)nc * N + lane, v);
            part = SYM_CONST | nc;
            ++nc;
            pw = 8u * run;
        } else {
            const uint32_t t = (tag - 1u) >> 5, j0 = (tag - 1u) & 31u;
            const uint32_t w = S.node[(size_t)t * N + lane].x >> 8;
            uint32_t run = 1u;
            ++k;
            if (w != 8u) {
                while (k < len && j0 + run <= 31u) {
                    const uint32_t q = off + k;
                    if (q >= msize || mtag_at(S, N, lane, q) != tag + run) break;
                    ++run;
                    ++k;
                }
            }
            if (w == 8u || run == 32u) {
                part = t;
                pw = w == 8u ? 8u : 256u;
            } else {
                const uint32_t hi = 255u - 8u * j0, lo = 248u - 8u * (j0 + run - 1u);
                uint32_t et;
                if (!sym_node_push(S, N, lane, SYM_EXTRACT | ((hi - lo + 1u) << 8), t, 0u, (hi << 16) | lo, nn, et))
                    return false;
                part = et - 1u;
                pw = hi - lo + 1u;
            }
        }
        if (acc == SYM_NONE) {
            acc = part;
            accw = pw;
        } else {
            uint32_t ct;
            if (!sym_node_push(S, N, lane, SYM_CONCAT | ((accw + pw) << 8), acc, part, accw | (pw << 16), nn, ct))
                return false;
            acc = ct - 1u;
            accw += pw;
        }
    }
    ref = acc;
    return true;
}

// binary ALU opcodes with symbolic semantics; compares push Bools (width 1)
DEV bool sym_bin_ok(uint32_t op) {
    return (op >= 0x01u && op <= 0x07u) || (op >= 0x10u && op <= 0x14u) || (op >= 0x16u && op <= 0x18u) ||
           (op >= 0x1au && op <= 0x1du);
}
DEV bool sym_is_cmp(uint32_t op) { return op >= 0x10u && op <= 0x14u; }
// environment word of an env opcode (MG_ENV_*), or 5 when none
DEV uint32_t sym_env_word(uint32_t op) {
    switch (op) {
    case 0x30: return 0u;   // ADDRESS
    case 0x33: return 1u;   // CALLER
    case 0x32: return 2u;   // ORIGIN
    case 0x34: return 3u;   // CALLVALUE
    case 0x3a: return 4u;   // GASPRICE
    default: return 5u;
    }
}


#define LANE_TAINT 2048u
#define ESC_TAINT 9u
#define TOBJ0 7u                  // MG_TAINT_OBJ0
#define T_POST 16u
#define T_EXPCOND 32u
#define T_YCLASS 64u
#define TREC_WORDS (MG_REC_HEADER + 11u)
#define T_IFLANE (1u << 24)
DEV uint32_t hrec_words(uint32_t n) { return MG_REC_HEADER + 8u * (n - 1u) + 3u; }

DEV uint32_t t_obj(const DevTaint &T, size_t N, uint32_t lane, uint32_t slot) {
    return T.sobj[(size_t)slot * N + lane];
}
DEV void t_set_obj(const DevTaint &T, size_t N, uint32_t lane, uint32_t slot, uint32_t h) {
    T.sobj[(size_t)slot * N + lane] = h;
}
DEV unsigned long long t_mask(const DevTaint &T, size_t N, uint32_t lane, uint32_t h) {
    return h ? T.omask[(size_t)h * N + lane] : 0ull;
}
DEV uint32_t t_new(const DevTaint &T, size_t N, uint32_t lane, uint32_t &nobj, unsigned long long m) {
    const uint32_t h = nobj++;
    T.omask[(size_t)h * N + lane] = m;
    return h;
}
// handle compaction: objects no stack slot holds any more are dropped and the
// device's own handles [fixed, nobj) renumbered in order (new <= old, so the
// masks move down in place); the host's handles and the environment's stay put
DEV void t_gc(const DevTaint &T, size_t N, uint32_t lane, uint32_t sp, uint32_t fixed, uint32_t &nobj) {
    uint32_t *__restrict__ rm = T.oremap + lane;
    for (uint32_t h = fixed; h < nobj; ++h) rm[(size_t)h * N] = 0u;
    for (uint32_t s = 0; s < sp; ++s) {
        const uint32_t h = t_obj(T, N, lane, s);
        if (h >= fixed) rm[(size_t)h * N] = 1u;
    }
    uint32_t next = fixed;
    for (uint32_t h = fixed; h < nobj; ++h) {
        if (!rm[(size_t)h * N]) continue;
        if (next != h) T.omask[(size_t)next * N + lane] = T.omask[(size_t)h * N + lane];
        rm[(size_t)h * N] = next++;
    }
    for (uint32_t s = 0; s < sp; ++s) {
        const uint32_t h = t_obj(T, N, lane, s);
        if (h >= fixed) t_set_obj(T, N, lane, s, rm[(size_t)h * N]);
    }
    nobj = next;
}
// MG_REC_ANNOT: [kind][atom][step][stack[-1]][stack[-2]][pc][op | post << 8]
DEV void rec_annot(const DevLanes &L, uint32_t lane, uint32_t at, uint32_t atom, uint32_t step, const U256 &v0,
                   const U256 &v1, uint32_t pc, uint32_t opw, uint32_t fent) {
    at = rec_head(L, lane, at, MG_REC_ANNOT, atom, step, v0);
    uint32_t *__restrict__ q = L.rec + lane;
    const size_t N = L.N;
#pragma unroll
    for (int k = 0; k < 8; ++k) q[(size_t)(at + k) * N] = v1.w[k];
    q[(size_t)(at + 8u) * N] = pc;
    q[(size_t)(at + 9u) * N] = opw;
    q[(size_t)(at + 10u) * N] = fent;
}
// MG_REC_HOOK: [kind][n][step][stack[-1]][stack[-2..-n]][pc][op][fent]
DEV void rec_hook(const DevLanes &L, const LaneView &V, uint32_t lane, uint32_t at, uint32_t n, uint32_t step,
                  uint32_t sp, uint32_t pc, uint32_t op, uint32_t fent) {
    at = rec_head(L, lane, at, MG_REC_HOOK, n, step, V.stack(sp - 1u));
    uint32_t *__restrict__ q = L.rec + lane;
    const size_t N = L.N;
    for (uint32_t j = 1u; j < n; ++j) {
        const U256 w = V.stack(sp - 1u - j);
#pragma unroll
        for (int k = 0; k < 8; ++k) q[(size_t)(at + 8u * (j - 1u) + k) * N] = w.w[k];
    }
    at += 8u * (n - 1u);
    q[(size_t)at * N] = pc;
    q[(size_t)(at + 1u) * N] = op;
    q[(size_t)(at + 2u) * N] = fent;
}
// Annotation set of the word an executed opcode pushes (instructions.py:330-1060
// with bitvec.py's unions): the operands' union for the ALU -- nothing for a
// concrete zero divisor (DIV/SDIV/MOD/SMOD push a fresh 0) or a BYTE index past
// the word, only the value's for BYTE (its index is made concrete) -- and a
// fresh object for every other push.  a, b = stack[-1], stack[-2] before.
DEV unsigned long long t_result_mask(const DevTaint &T, size_t N, uint32_t lane, uint32_t op, uint32_t sp0,
                                     const U256 &a, const U256 &b, bool b_sym) {
    const auto m = [&](uint32_t k) { return sp0 > k ? t_mask(T, N, lane, t_obj(T, N, lane, sp0 - 1u - k)) : 0ull; };
    switch (op) {
    case 0x01: case 0x02: case 0x03: case 0x0a: case 0x0b:
    case 0x10: case 0x11: case 0x12: case 0x13: case 0x14:
    case 0x16: case 0x17: case 0x18: case 0x1b: case 0x1c: case 0x1d:
        return m(0) | m(1);
    case 0x04: case 0x05: case 0x06: case 0x07:
        return (!b_sym && u_iszero(b)) ? 0ull : (m(0) | m(1));
    case 0x08: case 0x09:
        return m(0) | m(1) | m(2);
    case 0x15: case 0x19:
        return m(0);
    case 0x1a:
        return (u_fits32(a) && a.w[0] < 32u) ? m(1) : 0ull;
    default:
        return 0ull;
    }
}
// The taint effects of one executed instruction, in the reference's order: the
// pre-hook's annotate() on its operand object, the sink hook's collection,
// the mutator's push (a new object, the DUP'd object, the environment word's
// object), the post-hook's annotate() on the pushed object.
DEV void t_commit(const DevTaint &T, size_t N, uint32_t lane, uint32_t op, uint32_t kind, uint32_t tact,
                  uint32_t sp0, uint32_t nsp, uint32_t nin, bool pushes, bool symcd, const U256 &a, const U256 &b,
                  bool b_sym, unsigned long long pre_bit, unsigned long long post_bit, uint32_t &nobj,
                  unsigned long long &sink, uint32_t &tf) {
    const uint32_t pre_k = tact & 15u, sink_k = (tact >> 8) & 15u;
    if (pre_bit) {
        const uint32_t slot = sp0 - pre_k;
        uint32_t h = t_obj(T, N, lane, slot);
        if (!h) { h = t_new(T, N, lane, nobj, 0ull); t_set_obj(T, N, lane, slot, h); }
        T.omask[(size_t)h * N + lane] |= pre_bit;
    }
    if (sink_k && sp0 >= sink_k) {
        sink |= t_mask(T, N, lane, t_obj(T, N, lane, sp0 - sink_k));
        tf |= 1u;
    }
    if (kind == K_DUP) {
        const uint32_t src = sp0 - nin;
        uint32_t h = t_obj(T, N, lane, src);
        if (!h) { h = t_new(T, N, lane, nobj, 0ull); t_set_obj(T, N, lane, src, h); }
        t_set_obj(T, N, lane, sp0, h);
    } else if (kind == K_SWAP) {
        const uint32_t x = t_obj(T, N, lane, sp0 - 1u), y = t_obj(T, N, lane, sp0 - nin);
        t_set_obj(T, N, lane, sp0 - 1u, y);
        t_set_obj(T, N, lane, sp0 - nin, x);
    } else if (pushes) {
        uint32_t h = 0u;
        const uint32_t envw = sym_env_word(op);
        if (envw < 5u) h = envw + 1u;                     // environment.address/sender/... object
        else if (op == 0x36u && symcd) h = 6u;            // SymbolicCalldata.calldatasize object
        else {
            const unsigned long long rm = t_result_mask(T, N, lane, op, sp0, a, b, b_sym);
            if (rm) h = t_new(T, N, lane, nobj, rm);
        }
        t_set_obj(T, N, lane, nsp - 1u, h);
    }
    if (post_bit && nsp >= 1u) {
        uint32_t h = t_obj(T, N, lane, nsp - 1u);
        if (!h) { h = t_new(T, N, lane, nobj, 0ull); t_set_obj(T, N, lane, nsp - 1u, h); }
        T.omask[(size_t)h * N + lane] |= post_bit;
    }
}

__global__ __launch_bounds__(256) void k_sym_step(DevLanes L, DevSym S, DevTaint T, const DevCode *__restrict__ codes,
                                                  const uint8_t *__restrict__ a8,
                                                  const uint32_t *__restrict__ a32,
                                                  uint64_t m0, uint64_t m1, uint64_t m2, uint64_t m3,
                                                  uint32_t max_steps, uint32_t max_depth, uint32_t horizon,
                                                  uint32_t loop_bound, DevCounters *__restrict__ ctr,
                                                  uint32_t lanes_pb, unsigned long long *__restrict__ prof) {
    __shared__ uint32_t s_kc[(256u / 64u) * KC_WAVE];
    if ((threadIdx.x & 63u) < 2u) s_kc[(threadIdx.x >> 6) * KC_WAVE + KC_E * 24u + (threadIdx.x & 63u)] = 0u;
    __syncthreads();
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= L.n || L.status[lane] != ST_RUNNING) return;
    const uint32_t flags = L.flags[lane];
    if (!(flags & (LANE_SYMBOLIC | LANE_TAINT))) return;
    uint32_t lflags = flags;                 // + LANE_MEMTAG once a symbolic byte is written
    const size_t N = L.N;
    // symbolic semantics need the arena planes; taint needs the taint planes
    const bool symlane = (flags & LANE_SYMBOLIC) && S.stag != nullptr;
    const bool tl = (flags & LANE_TAINT) && T.sobj != nullptr;
    const DevCode C = codes[L.code_id[lane]];
    const uint8_t *__restrict__ gops = a8 + C.op_off;
    const uint8_t *__restrict__ gfent = a8 + C.fent_off;
    uint32_t pc = L.pc[lane], sp = L.sp[lane], msize = L.msize[lane], depth = L.depth[lane];
    uint32_t fent = L.fent[lane];
    uint64_t gmin = L.gas_min[lane], gmax = L.gas_max[lane];
    const uint64_t txlim = L.gas_limit[lane];
    const uint64_t glim = txlim < MSTATE_GAS_LIMIT + 1ull ? txlim : MSTATE_GAS_LIMIT + 1ull;
    uint32_t nn = symlane ? S.n_nodes[lane] : 0u, nc = symlane ? S.n_consts[lane] : 0u;
    uint32_t nobj = 0u, tfixed = 0u, natoms = 0u, ttf = 0u;
    unsigned long long tsink = 0ull, tym = 0ull;
    if (tl) {
        nobj = T.n_obj[lane]; tfixed = T.n_fixed[lane]; natoms = T.n_atoms[lane]; ttf = T.tflags[lane];
        tsink = T.sink[lane]; tym = T.ymask[lane];
    }
    const bool hook_ack = (flags & LANE_HOOK_ACK) != 0u;
    const bool creation = (flags & LANE_CREATION) != 0u;
    uint32_t lane_max = (flags & LANE_STEP1) ? min(max_steps, 1u) : max_steps;
    if (horizon) {
        const uint32_t s0 = L.steps[lane];
        lane_max = min(lane_max, horizon > s0 ? horizon - s0 : 0u);
    }
    uint32_t status = ST_RUNNING, aux = 0u, executed = 0u, n_sha3 = 0u, n_exp = 0u;
    const bool loop_on = loop_bound != 0u && L.trace_cap != 0u;
    uint32_t tlen = loop_on ? L.trace_len[lane] : 0u;
    const LaneView V{L, lane, nullptr, 0u, threadIdx.x, 256u, nullptr, 0u};
    const StepEnv E{&L, C, a8, a32, nullptr, nullptr, nullptr, nullptr, nullptr,
                    s_kc + (threadIdx.x >> 6) * KC_WAVE, txlim, glim, lane, threadIdx.x, 256u, 0u, flags,
                    0u, 0u, 0u, 0u, 0u, 1u};

    // optional opcode histogram (mg_step_profile; profiling passes only): the
    // previous instruction is counted once `executed` shows it completed
    uint32_t pexec = 0u, pop = 0u;
    for (;;) {
        if (prof && executed != pexec) { atomicAdd(&prof[pop], 1ull); pexec = executed; }
        // the checks svm.execute_state makes before an instruction (svm.py:369-402)
        if (max_depth != 0u && depth >= max_depth) { status = ST_DEPTH; break; }
        if (pc >= C.n_instr) { status = ST_END; break; }
        const uint32_t op = gops[pc];
        pop = op;
        const uint2 d = kDec[op];
        const uint32_t kind = (d.y >> 9) & 31u;
        const uint64_t hm = op < 64u ? m0 : op < 128u ? m1 : op < 192u ? m2 : m3;
        const bool acked = hook_ack && executed == 0u;     // the host ran this instruction's hooks
        const bool hooked = ((hm >> (op & 63u)) & 1ull) && !acked;
        if (loop_on && !acked && (hooked || executed < lane_max)) {
            // BoundedLoopsStrategy: every instruction the path is popped at, as k_lane_step
            const uint64_t tr = trace_step(L.trace, N, L.trace_cap, lane, tlen, a32[C.addr_off + pc], op == 0x5bu,
                                           loop_bound, creation ? 1u : 0u);
            tlen = (uint32_t)tr;
            const uint32_t res = (uint32_t)(tr >> 60);
            if (res == 1u) { status = ST_LOOP; aux = (uint32_t)(tr >> 32) & 0x0fffffffu; break; }
            if (res == 2u) { status = ST_ESCAPE; aux = op | (ESC_TRACE << 8); break; }
        }
        if (hooked) { status = ST_HOOK; aux = op; break; }
        if (executed >= lane_max) break;
        const uint32_t uy = op | (d.y << 8) | pd_flags(op, d.y, 0u) | ((uint32_t)gfent[pc] << 22);
        // a creation's calldata opcodes run here on a lane with symbolic calldata (below)
        if (((uy & PD_SPECIAL) &&
             !(((op == 0x47u && (flags & LANE_SYMBAL) && symlane) || (op == 0x31u && (flags & LANE_BALANCE) && symlane) ||
                ((op == 0x5au || op == 0x41u || op == 0x42u || op == 0x44u) && symlane) ||
                ((op == 0x43u || op == 0x46u) && (flags & LANE_SYMBLOCK) && symlane)) && !tl)) ||
            // a creation's CODESIZE / CODECOPY / CALLDATA* run below only on a
            // symbolic-calldata lane without taint (the block that implements them
            // skips taint lanes); anywhere else the host steps them
            (creation && (uy & PD_CREATION) && !(symlane && (flags & LANE_SYMCD) && !tl))) {
            status = ST_ESCAPE; aux = op | (ESC_OPCODE << 8); break;
        }
        const uint32_t req = d.y & 15u, npop = (d.y >> 4) & 15u;
        const bool pushes = ((d.y >> 8) & 1u) != 0u;
        uint32_t nin = npop;                        // stack words the instruction reads
        if (kind == K_DUP) nin = op - 0x7fu;
        else if (kind == K_SWAP) nin = op - 0x8fu + 1u;
        bool any_sym = false;
        if (symlane)
            for (uint32_t k = 0; k < nin && k < sp; ++k) any_sym |= sym_tag(S, N, lane, sp - 1u - k) != 0u;
        const uint32_t envw = sym_env_word(op);
        const bool env_sym = symlane && envw < 5u && ((flags >> (LANE_SYMENV_SHIFT + envw)) & 1u);
        const bool cd_sym = symlane && (flags & LANE_SYMCD) && (op == 0x35u || op == 0x36u || op == 0x37u);
        const bool stack_op = kind == K_DUP || kind == K_SWAP || kind == K_POP;

        // ---- taint lanes: this opcode's batch-safe hooks (mythril_amd/laser/taint.py) ----
        uint32_t tact = (tl && !acked) ? T.prog[op] : 0u;
        unsigned long long pre_bit = 0ull, post_bit = 0ull;
        uint32_t rec_save = 0u;
        bool rec_pre = false;
        // an address modules have cached an issue at: their hooks return early there
        // (base.py:79-86): 2 = all of this opcode's modules (no actions), 1 = some
        // of them (the host runs the hooks)
        if (tact && T.force) {
            const uint8_t f = T.force[C.cov_off + pc];
            if (f == 1u) { status = ST_HOOK; aux = op; break; }
            if (f == 2u) tact = 0u;
        }
        if (tact) {
            const uint32_t yk = (tact >> 12) & 15u, pre_k = tact & 15u;
            const uint32_t dk = (tact >> 16) & 15u, sk = (tact >> 20) & 15u;
            // a yield-if hook has work only when its operand carries an atom of the class
            if (yk && sp >= yk && (t_mask(T, N, lane, t_obj(T, N, lane, sp - yk)) & tym)) {
                status = ST_HOOK; aux = op; break;
            }
            // hooks with work only on a symbolic operand, or on lanes whose state
            // carries a given annotation; a deferred hook's words must be concrete
            bool ysym = false;
            if (symlane) {
                if (sk && sp >= sk && sym_tag(S, N, lane, sp - sk)) ysym = true;
                for (uint32_t j = 0; j < dk && j < sp; ++j) ysym |= sym_tag(S, N, lane, sp - 1u - j) != 0u;
            }
            if (ysym || ((tact & T_IFLANE) && (ttf & 2u))) { status = ST_HOOK; aux = op; break; }
            bool do_pre = pre_k != 0u && sp >= pre_k && sp >= req;
            const bool do_post = (tact & T_POST) != 0u;
            if (do_pre || do_post) {
                // the device replays annotating hooks on concrete words only; the host
                // runs them (MG_HOOK) on symbolic ones and around SHA3/EXP results
                if (any_sym || env_sym || cd_sym || (do_post && (kind == K_SHA3 || op == 0x0au))) {
                    status = ST_HOOK; aux = op; break;
                }
                if (do_pre && (tact & T_EXPCOND)) {
                    // integer.py:161-166: no annotation for exponent 0 or base < 2
                    const U256 base = V.stack(sp - 1u);
                    const U256 ex = sp >= 2u ? V.stack(sp - 2u) : u_zero();
                    if (u_iszero(ex) || (u_fits32(base) && base.w[0] < 2u)) do_pre = false;
                }
            }
            const uint32_t need = (do_pre ? 1u : 0u) + (do_post ? 1u : 0u);
            const bool defer = dk != 0u && sp >= dk;
            if (natoms + need > 64u) { status = ST_ESCAPE; aux = op | (ESC_TAINT << 8); break; }
            if (nobj + 4u > T.obj_cap) {
                t_gc(T, N, lane, sp, tfixed, nobj);
                if (nobj + 4u > T.obj_cap) { status = ST_ESCAPE; aux = op | (ESC_TAINT << 8); break; }
            }
            if ((need || defer) && (uint64_t)L.rec_len[lane] + need * TREC_WORDS + (defer ? hrec_words(dk) : 0u) >
                                       L.rec_cap) {
                status = ST_ESCAPE; aux = op | (ESC_RECORD << 8); break;
            }
            rec_save = L.rec_len[lane];
            if (do_pre) {
                // logged before the mutator runs: its own records (EXP) follow
                rec_annot(L, lane, L.rec_len[lane], natoms, L.steps[lane] + executed, V.stack(sp - 1u),
                          sp >= 2u ? V.stack(sp - 2u) : u_zero(), pc, op, fent);
                L.rec_len[lane] += TREC_WORDS;
                rec_pre = true;
                pre_bit = 1ull << natoms;
            }
            if (defer) {
                // the deferred hook runs after the annotating ones of the opcode, as
                // the host replays records in log order
                rec_hook(L, V, lane, L.rec_len[lane], dk, L.steps[lane] + executed, sp, pc, op, fent);
                L.rec_len[lane] += hrec_words(dk);
                rec_pre = true;
            }
            if (do_post) post_bit = 1ull << (natoms + (do_pre ? 1u : 0u));
        } else if (tl && nobj + 4u > T.obj_cap) {
            t_gc(T, N, lane, sp, tfixed, nobj);
            if (nobj + 4u > T.obj_cap) { status = ST_ESCAPE; aux = op | (ESC_TAINT << 8); break; }
        }

        // ---- symbolic calldata into memory, and a creation's calldata opcodes ----
        // CALLDATACOPY of symbolic calldata (_calldata_copy_helper,
        // instructions.py:807-875): memory byte mstart + k becomes calldata[dstart + k],
        // one CDBYTE node per byte tagged into memory; size 0 copies and extends
        // nothing.  In a creation transaction (instructions.py:878-891, 979-1000,
        // 1074-1104) CALLDATACOPY pops its operands and copies nothing, CODESIZE is
        // the code's size + 0x200 with `calldata.size == it` appended to the path
        // (MG_REC_CDSIZE, replayed by the host in execution order), and CODECOPY from
        // at or past the end of the code is that calldata copy at code_offset minus
        // the code's size.  A message call's CALLDATACOPY with a symbolic memory offset
        // copies nothing and one with a symbolic size copies 320 bytes, as the
        // reference does; a symbolic calldata offset stays with the host.
        if (symlane && (flags & LANE_SYMCD) && !tl && sp >= max(req, npop) &&
            (op == 0x37u || (creation && op == 0x38u) ||
             (creation && op == 0x39u && !sym_tag(S, N, lane, sp - 2u) &&
              !(u_fits32(V.stack(sp - 2u)) && V.stack(sp - 2u).w[0] < C.n_bytes)))) {
            const uint64_t gtmin = d.x & 0xffffu, gtmax = d.x >> 16;
            uint32_t nsp = sp - npop, nmsize = msize, lnn = nn, stop = ST_RUNNING, sx = 0u, rec_new = 0u;
            uint64_t ngmin = gmin, ngmax = gmax;
            U256 rval = u_zero();
            bool wrote_tag = false;
            do {
#define CSTOPX(s_, x_) { stop = (s_); sx = (x_); break; }
                if (op == 0x38u) {                                   // creation CODESIZE
                    if (nsp + 1u > STACK_LIMIT) CSTOPX(ST_VMEXC, EXC_OVERFLOW)
                    if (nsp + 1u > L.stack_cap) CSTOPX(ST_ESCAPE, op | (ESC_STACK << 8))
                    const uint32_t rec_at = L.rec_len[lane];
                    if (!L.rec_cap || (uint64_t)rec_at + MG_REC_HEADER > L.rec_cap)
                        CSTOPX(ST_ESCAPE, op | (ESC_RECORD << 8))
                    ngmin += gtmin; ngmax += gtmax;
                    if (ngmin >= glim) CSTOPX(ST_VMEXC, EXC_OOG)
                    rval = u_small(C.n_bytes + 0x200u);
                    rec_new = rec_head(L, lane, rec_at, MG_REC_CDSIZE, 0u, L.steps[lane] + executed, rval);
                    break;
                }
                if (creation && op == 0x37u) {                       // creation CALLDATACOPY: pops only
                    ngmin += gtmin; ngmax += gtmax;
                    if (ngmin >= glim) CSTOPX(ST_VMEXC, EXC_OOG)
                    break;
                }
                const uint32_t ta = sym_tag(S, N, lane, sp - 1u), tb = sym_tag(S, N, lane, sp - 2u);
                uint32_t tc = sym_tag(S, N, lane, sp - 3u);
                U256 a = V.stack(sp - 1u), b = V.stack(sp - 2u), c = V.stack(sp - 3u);
                if (op == 0x37u && ta) {
                    // a symbolic memory offset: the copy is dropped (instructions.py:810-814)
                    ngmin += gtmin; ngmax += gtmax;
                    if (ngmin >= glim) CSTOPX(ST_VMEXC, EXC_OOG)
                    break;
                }
                // a symbolic size copies SYMBOLIC_CALLDATA_SIZE bytes (instructions.py:822-826,
                // call.py:33); a symbolic calldata offset y makes byte k calldata[y + k]
                const bool symsrc = op == 0x37u && tb != 0u;
                if (op == 0x37u && tc) { c = u_small(320u); tc = 0u; }
                if (ta || (tb && !symsrc) || tc) CSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                if (u_iszero(c)) {                                   // size 0: nothing but the gas
                    ngmin += gtmin; ngmax += gtmax;
                    if (ngmin >= glim) CSTOPX(ST_VMEXC, EXC_OOG)
                    break;
                }
                const int mx = mem_extend(a, c, nmsize, ngmin, ngmax, L.mem_cap, (int64_t)gtmin, txlim);
                if (mx == MX_OOG) CSTOPX(ST_VMEXC, EXC_OOG)
                if (mx == MX_ESCAPE) CSTOPX(ST_ESCAPE, op | (ESC_MEMORY << 8))
                ngmin += gtmin; ngmax += gtmax;
                if (ngmin >= glim) CSTOPX(ST_VMEXC, EXC_OOG)
                // the source index of every byte must stay below 2^32 on the device
                const uint32_t src = op == 0x39u ? b.w[0] - C.n_bytes : b.w[0];
                const uint32_t size = c.w[0], mst = a.w[0];
                if (!symsrc && (!u_fits32(b) || (uint64_t)src + size > 0xffffffffull))
                    CSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                if ((uint64_t)lnn + size > S.node_cap) CSTOPX(ST_ESCAPE, op | (ESC_ARENA << 8))
                if (nmsize > msize) V.mzero(msize, nmsize);
                for (uint32_t k = 0; k < size; ++k) {
                    uint32_t tg;
                    if (symsrc) sym_node_push(S, N, lane, SYM_CDBYTEX | (8u << 8), tb - 1u, 0u, k, lnn, tg);
                    else sym_node_push(S, N, lane, SYM_CDBYTE | (8u << 8), 0u, 0u, src + k, lnn, tg);
                    V.set_mbyte(mst + k, 0u);
                    set_mtag(S, N, lane, mst + k, 1u + (((tg - 1u) << 5) | 31u));
                }
                wrote_tag = true;
#undef CSTOPX
            } while (0);
            if (stop != ST_RUNNING) {
                if (stop != ST_ESCAPE) ++executed;
                status = stop; aux = sx; break;
            }
            if (rec_new) L.rec_len[lane] = rec_new;
            if (wrote_tag) lflags |= LANE_MEMTAG;
            if (op == 0x38u) {
                V.set_stack(nsp, rval);
                sym_set_tag(S, N, lane, nsp, 0u);
                ++nsp;
            }
            sp = nsp; ++pc; msize = nmsize; gmin = ngmin; gmax = ngmax; nn = lnn;
            ++executed;
            continue;
        }

        // ---- symbolic lanes: storage chain, memory byte tags, symbolic SHA3 ----
        // (instructions.py:1013-1051, 1437-1518; account.py:43-87; memory.py:56-115).
        // Storage of a symbolic lane is the reference's store chain (one entry per
        // SSTORE), so every SLOAD / SSTORE runs here; memory operations run here
        // when a byte they read is symbolic or the word they write is, or to clear
        // the tags of bytes a concrete write replaces.
        bool memlane = false;
        const bool memop = kind == K_SLOAD || kind == K_SSTORE || kind == K_MLOAD || kind == K_MSTORE ||
                           kind == K_MSTORE8 || kind == K_SHA3;      // each pops >= 1 word
        if (symlane && memop && sp >= max(max(req, npop), 1u)) {
            const uint32_t ta0 = sym_tag(S, N, lane, sp - 1u);
            const uint32_t tb0 = npop >= 2u ? sym_tag(S, N, lane, sp - 2u) : 0u;
            if (kind == K_SLOAD || kind == K_SSTORE) memlane = true;
            else if (kind == K_MLOAD || kind == K_MSTORE || kind == K_MSTORE8)
                memlane = ta0 != 0u || tb0 != 0u || (lflags & LANE_MEMTAG);
            else if (kind == K_SHA3) {
                const U256 a0 = V.stack(sp - 1u), b0 = V.stack(sp - 2u);
                memlane = ta0 != 0u || tb0 != 0u ||
                          ((lflags & LANE_MEMTAG) && u_fits32(a0) && u_fits32(b0) && b0.w[0] != 0u &&
                           mtag_any(S, N, lane, a0.w[0], b0.w[0], msize));
            }
        }
        if (memlane) {
            const uint32_t ta = sym_tag(S, N, lane, sp - 1u);
            const uint32_t tb = npop >= 2u ? sym_tag(S, N, lane, sp - 2u) : 0u;
            const U256 a = V.stack(sp - 1u);
            const U256 b = npop >= 2u ? V.stack(sp - 2u) : u_zero();
            const uint32_t nsp = sp - npop;
            uint32_t lnn = nn, lnc = nc, rtag = 0u, nmsize = msize, rec_new = 0u, stop = ST_RUNNING, sx = 0u;
            uint64_t ngmin = gmin, ngmax = gmax;
            U256 rval = u_zero();
            bool wrote_tag = false;
            const uint64_t gtmin = d.x & 0xffffu, gtmax = d.x >> 16;
            // a taint lane's annotating hooks on these opcodes run on the host, and
            // symbolic memory words carry annotation sets the lane does not track
            const bool tbusy = tl && (pre_bit != 0ull || post_bit != 0ull);
            const bool memsym = kind != K_SLOAD && kind != K_SSTORE;
            do {
                if (tbusy) { stop = ST_HOOK; sx = op; break; }
#define MSTOPX(s_, x_) { stop = (s_); sx = (x_); break; }
#define MGAS() { ngmin += gtmin; ngmax += gtmax; if (ngmin >= glim) MSTOPX(ST_VMEXC, EXC_OOG) }
#define MPUSHCHK() { if (nsp + 1u > STACK_LIMIT) MSTOPX(ST_VMEXC, EXC_OVERFLOW) \
                     if (nsp + 1u > L.stack_cap) MSTOPX(ST_ESCAPE, op | (ESC_STACK << 8)) }
#define MMEMX(st_, sz_, later_) { const int mx_ = mem_extend((st_), (sz_), nmsize, ngmin, ngmax, L.mem_cap, \
                                                             (later_), txlim); \
                                  if (mx_ == MX_OOG) MSTOPX(ST_VMEXC, EXC_OOG) \
                                  if (mx_ == MX_ESCAPE) MSTOPX(ST_ESCAPE, op | (ESC_MEMORY << 8)) }
                if (memsym && ta) {
                    // a symbolic offset: the reference keys its byte map by simplify(index)
                    // (memory.py:117-203).  MSTORE / MSTORE8 append an event node (offset,
                    // value, kind) to the arena and MLOAD makes an MLOADK node; the host
                    // decodes both by replaying the events into that byte map, so no key
                    // equality is decided here.  No extension and no memory gas
                    // (mem_extend returns on a symbolic start, machine_state.py:171-180).
                    // SHA3 of a concrete length reads the same way: an MLOADK node over
                    // [offset, offset + length) feeds a KECCAK node (sha3_, instructions.py:
                    // 1014-1051).  A symbolic or zero length and taint lanes stay with the host.
                    if (tl) MSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                    if (kind == K_SHA3) {
                        if (tb || !u_fits32(b) || b.w[0] == 0u || b.w[0] > 4096u)
                            MSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                        const uint32_t len = b.w[0];
                        if (!L.rec_cap) MSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                        const uint64_t g = 30ull + 6ull * (((uint64_t)len + 31ull) >> 5);
                        ngmin += g; ngmax += g;
                        if (ngmin >= glim) MSTOPX(ST_VMEXC, EXC_OOG)
                        const uint32_t rec_at = L.rec_len[lane];
                        if ((uint64_t)rec_at + MG_REC_HEADER + 1u > L.rec_cap)
                            MSTOPX(ST_ESCAPE, op | (ESC_RECORD << 8))
                        MPUSHCHK()
                        uint32_t mt;
                        if (!sym_node_push(S, N, lane, SYM_MLOADK | ((8u * len) << 8), ta - 1u, 0u, len, lnn, mt) ||
                            !sym_node_push(S, N, lane, SYM_KECCAK | (256u << 8), mt - 1u, 0u, 8u * len, lnn, rtag))
                            MSTOPX(ST_ESCAPE, op | (ESC_ARENA << 8))
                        rec_new = rec_head(L, lane, rec_at, MG_REC_SYMKECCAK, len, L.steps[lane] + executed, u_zero());
                        L.rec[(size_t)rec_new * N + lane] = rtag - 1u;
                        ++rec_new;
                        ++n_sha3;
                    } else if (kind == K_MLOAD) {
                        MPUSHCHK()
                        MGAS()
                        if (!sym_node_push(S, N, lane, SYM_MLOADK | (256u << 8), ta - 1u, 0u, 0u, lnn, rtag))
                            MSTOPX(ST_ESCAPE, op | (ESC_ARENA << 8))
                    } else {
                        MGAS()
                        uint32_t vref, et;
                        if (!sym_ref(S, N, lane, tb, b, lnc, vref) ||
                            !sym_node_push(S, N, lane, SYM_MSTOREK, ta - 1u, vref, kind == K_MSTORE8 ? 2u : 1u,
                                           lnn, et))
                            MSTOPX(ST_ESCAPE, op | (ESC_ARENA << 8))
                    }
                    break;
                }
                if (kind == K_SLOAD) {
                    // simplify(Select(chain, index)): from the newest store, the same
                    // index term answers, a distinct constant index (both constant) is
                    // skipped, anything else stops the walk (expr._select)
                    const uint32_t cnt = L.storage_count[lane];
                    int32_t e = (int32_t)cnt - 1;
                    bool hit = false;
                    for (; e >= 0; --e) {
                        const uint2 tg = S.sttag[(size_t)e * N + lane];
                        if (!ta && !tg.x) {
                            if (u_eq(ld_word(gv(L.storage), V.row((uint32_t)e) * 2), a)) { hit = true; break; }
                            continue;
                        }
                        if (ta && tg.x && sym_same(S.node, S.cval, N, lane, ta - 1u, tg.x - 1u)) hit = true;
                        break;
                    }
                    MPUSHCHK()
                    MGAS()
                    if (hit) {
                        const uint2 tg = S.sttag[(size_t)e * N + lane];
                        if (tg.y) rtag = tg.y;
                        else rval = ld_word(gv(L.storage), V.row((uint32_t)e) * 2 + 1);
                    } else if (e < 0 && !(lflags & LANE_SYMSTORE)) {
                        rval = u_zero();                             // K(256, 256, 0): its default
                    } else {
                        uint32_t ya;
                        if (!sym_ref(S, N, lane, ta, a, lnc, ya) ||
                            !sym_node_push(S, N, lane, SYM_SLOAD | (256u << 8), ya, cnt, 0u, lnn, rtag))
                            MSTOPX(ST_ESCAPE, op | (ESC_ARENA << 8))
                    }
                } else if (kind == K_SSTORE) {
                    // a new Store on the chain (account.py:77-87), never in place
                    if (flags & LANE_STATIC) MSTOPX(ST_VMEXC, EXC_WRITEPROT)
                    const uint32_t cnt = L.storage_count[lane];
                    if (cnt >= L.storage_cap) MSTOPX(ST_ESCAPE, op | (ESC_STORAGE << 8))
                    MGAS()
                    st_word(gv(L.storage), V.row(cnt) * 2, ta ? u_zero() : a);
                    st_word(gv(L.storage), V.row(cnt) * 2 + 1, tb ? u_zero() : b);
                    S.sttag[(size_t)cnt * N + lane] = make_uint2(ta, tb);
                    L.storage_count[lane] = cnt + 1u;
                } else if (kind == K_MLOAD) {
                    MMEMX(a, u_small(32), (int64_t)gtmin)
                    MPUSHCHK()
                    MGAS()
                    if (nmsize > msize) V.mzero(msize, nmsize);
                    if ((lflags & LANE_MEMTAG) && mtag_any(S, N, lane, a.w[0], 32u, nmsize)) {
                        if (tl) MSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                        uint32_t r;
                        if (!sym_mem_ref(S, L.mem, N, lane, a.w[0], 32u, nmsize, lnn, lnc, r))
                            MSTOPX(ST_ESCAPE, op | (ESC_ARENA << 8))
                        rtag = r + 1u;
                    } else {
                        rval = V.mword(a.w[0]);
                    }
                } else if (kind == K_MSTORE || kind == K_MSTORE8) {
                    const bool m8 = kind == K_MSTORE8;
                    if (tb && tl) MSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                    MMEMX(a, u_small(m8 ? 1u : 32u), (int64_t)gtmin)
                    MGAS()
                    if (nmsize > msize) V.mzero(msize, nmsize);
                    const uint32_t off = a.w[0];
                    if (tb) {
                        // write_word_at: byte j = Extract(255 - 8j, 248 - 8j, value);
                        // MSTORE8: Extract(7, 0, value) (memory.py:102-115, instructions.py:1472-1493)
                        const uint32_t base = (tb - 1u) << 5;
                        if (m8) {
                            V.set_mbyte(off, 0u);
                            set_mtag(S, N, lane, off, 1u + (base | 31u));
                        } else {
                            V.set_mword(off, u_zero());
                            for (uint32_t j = 0; j < 32u; ++j) set_mtag(S, N, lane, off + j, 1u + (base | j));
                        }
                        wrote_tag = true;
                    } else {
                        if (m8) V.set_mbyte(off, b.w[0] & 0xffu);
                        else V.set_mword(off, b);
                        if (lflags & LANE_MEMTAG)
                            for (uint32_t j = 0; j < (m8 ? 1u : 32u); ++j) set_mtag(S, N, lane, off + j, 0u);
                    }
                } else {  // K_SHA3 over symbolic bytes: keccak256_<8 len>(data), create_keccak
                    if (tl) MSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                    // a symbolic length is taken as 64 with `length == 64` appended to the
                    // path (instructions.py:1023-1028, an MG_REC_SYMLEN record before the
                    // SHA3's own); only over a range holding a symbolic byte, so the data
                    // (and the hash) stay symbolic as in the reference
                    if (tb && (sym_width(S, N, lane, tb) == 1u || !u_fits32(a) ||
                               !((lflags & LANE_MEMTAG) && mtag_any(S, N, lane, a.w[0], 64u, msize))))
                        MSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                    const uint32_t len = tb ? 64u : b.w[0];
                    if (!L.rec_cap) MSTOPX(ST_ESCAPE, op | (ESC_SYMBOLIC << 8))
                    const uint64_t g = 30ull + 6ull * (((uint64_t)len + 31ull) >> 5);
                    ngmin += g; ngmax += g;
                    // the reference has appended the length constraint before this check:
                    // an out-of-gas SHA3 of a symbolic length is the host's
                    if (ngmin >= glim) MSTOPX(tb ? ST_ESCAPE : ST_VMEXC, tb ? op | (ESC_SYMBOLIC << 8) : EXC_OOG)
                    MMEMX(a, u_small(len), -1)
                    uint32_t rec_at = L.rec_len[lane];
                    const uint32_t rec_need = (tb ? MG_REC_HEADER + 1u : 0u) + MG_REC_HEADER + 1u;
                    if ((uint64_t)rec_at + rec_need > L.rec_cap) MSTOPX(ST_ESCAPE, op | (ESC_RECORD << 8))
                    if (tb) {
                        const uint32_t at = rec_head(L, lane, rec_at, MG_REC_SYMLEN, 64u, L.steps[lane] + executed,
                                                     u_zero());
                        L.rec[(size_t)at * N + lane] = tb - 1u;
                        rec_at = at + 1u;
                    }
                    if (nmsize > msize) V.mzero(msize, nmsize);
                    MPUSHCHK()
                    uint32_t r;
                    if (!sym_mem_ref(S, L.mem, N, lane, a.w[0], len, nmsize, lnn, lnc, r) ||
                        !sym_node_push(S, N, lane, SYM_KECCAK | (256u << 8), r, 0u, 8u * len, lnn, rtag))
                        MSTOPX(ST_ESCAPE, op | (ESC_ARENA << 8))
                    rec_new = rec_head(L, lane, rec_at, MG_REC_SYMKECCAK, len, L.steps[lane] + executed, u_zero());
                    L.rec[(size_t)rec_new * N + lane] = rtag - 1u;
                    ++rec_new;
                    ++n_sha3;
                }
#undef MSTOPX
#undef MGAS
#undef MPUSHCHK
#undef MMEMX
            } while (0);
            if (stop != ST_RUNNING) {
                if (rec_pre) L.rec_len[lane] = rec_save;   // the instruction did not run
                if (stop != ST_ESCAPE && stop != ST_HOOK) ++executed;
                status = stop; aux = sx; break;
            }
            if (rec_new) L.rec_len[lane] = rec_new;
            if (wrote_tag) lflags |= LANE_MEMTAG;
            if (tl)
                t_commit(T, N, lane, op, kind, tact, sp, nsp + (pushes ? 1u : 0u), nin, pushes, false, a, b, tb != 0u,
                         pre_bit, post_bit, nobj, tsink, ttf);
            if (pushes) {
                V.set_stack(nsp, rval);
                sym_set_tag(S, N, lane, nsp, rtag);
            }
            sp = nsp + (pushes ? 1u : 0u); ++pc; msize = nmsize; gmin = ngmin; gmax = ngmax; nn = lnn; nc = lnc;
            if (pre_bit) { ++natoms; if (tact & T_YCLASS) tym |= pre_bit; }
            ++executed;
            continue;
        }

        if (op == 0x47u || op == 0x5au || op == 0x41u || op == 0x42u || op == 0x44u || op == 0x43u || op == 0x46u ||
            (op == 0x3du && (flags & LANE_SYMRDS) && !tl)) {
            // SELFBALANCE on a lane whose balance is symbolic (selfbalance_,
            // instructions.py:968-976; taint lanes escaped above):
            // environment.active_account.balance(), the balances array at the active
            // address; RETURNDATASIZE after a host CALL that left a symbolic size
            // (returndatasize_, :1359-1370): last_return_data.size.  ENV nodes the
            // host decodes.  No host CALL runs inside a device run, so neither value
            // can move under it.
            // GAS, COINBASE, TIMESTAMP, DIFFICULTY on a symbolic lane (:1386-1425,
            // 1700-1709): the transaction's fresh variable of that name, new_bitvec;
            // NUMBER, CHAINID (:958-965, 1406-1413) when the environment holds them
            // symbolic (MG_LANE_SYMBLOCK): environment.block_number / chainid
            const uint32_t which = op == 0x47u ? MG_ENV_SELFBALANCE : op == 0x5au ? MG_ENV_GAS :
                                   op == 0x41u ? MG_ENV_COINBASE : op == 0x42u ? MG_ENV_TIMESTAMP :
                                   op == 0x44u ? MG_ENV_DIFFICULTY : op == 0x43u ? MG_ENV_NUMBER :
                                   op == 0x46u ? MG_ENV_CHAINID : MG_ENV_RETURNDATASIZE;
            const uint64_t ngmin = gmin + (d.x & 0xffffu), ngmax = gmax + (d.x >> 16);
            uint32_t lnn = nn, rtag = 0u;
            if (sp + 1u > STACK_LIMIT) { ++executed; status = ST_VMEXC; aux = EXC_OVERFLOW; break; }
            if (sp + 1u > L.stack_cap) { status = ST_ESCAPE; aux = op | (ESC_STACK << 8); break; }
            if (!sym_node_push(S, N, lane, SYM_ENV | (256u << 8), 0u, 0u, which, lnn, rtag)) {
                status = ST_ESCAPE; aux = op | (ESC_ARENA << 8); break;
            }
            if (ngmin >= glim) { ++executed; status = ST_VMEXC; aux = EXC_OOG; break; }
            V.set_stack(sp, u_zero());
            sym_set_tag(S, N, lane, sp, rtag);
            ++sp; ++pc; gmin = ngmin; gmax = ngmax; nn = lnn;
            ++executed;
            continue;
        }

        if (op == 0x31u) {   // (only on MG_LANE_BALANCE lanes; taint lanes escaped above)
            // BALANCE (balance_, instructions.py:907-931) with no dynamic loader: the
            // account's balance() for a known concrete address, else If(address ==
            // account.address, account.balance(), ...) over the world state's accounts.
            // A BALANCE node over the address; the host builds the term from the lane's
            // world state, which no device instruction changes.
            if (sp < 1u) { status = ST_ESCAPE; aux = op | (ESC_SYMBOLIC << 8); break; }   // the host's underflow
            const U256 a = V.stack(sp - 1u);
            const uint32_t ta = sym_tag(S, N, lane, sp - 1u);
            if (ta && sym_width(S, N, lane, ta) == 1u) { status = ST_ESCAPE; aux = op | (ESC_SYMBOLIC << 8); break; }
            const uint64_t ngmin = gmin + (d.x & 0xffffu), ngmax = gmax + (d.x >> 16);
            uint32_t lnn = nn, lnc = nc, ya = 0u, rtag = 0u;
            if (!sym_ref(S, N, lane, ta, a, lnc, ya) ||
                !sym_node_push(S, N, lane, SYM_BALANCE | (256u << 8), ya, 0u, 0u, lnn, rtag)) {
                status = ST_ESCAPE; aux = op | (ESC_ARENA << 8); break;
            }
            if (ngmin >= glim) { ++executed; status = ST_VMEXC; aux = EXC_OOG; break; }
            V.set_stack(sp - 1u, u_zero());
            sym_set_tag(S, N, lane, sp - 1u, rtag);
            ++pc; gmin = ngmin; gmax = ngmax; nn = lnn; nc = lnc;
            ++executed;
            continue;
        }

        if (any_sym && !tl && (kind == K_JUMP || (kind == K_JUMPI && sp >= 2u)) && sp >= 1u &&
            sym_never_const(S, N, lane, sym_tag(S, N, lane, sp - 1u))) {
            // a symbolic jump target: JUMP raises InvalidJumpDestination (jump_,
            // instructions.py:1529-1532), a VmException at the instruction's start;
            // JUMPI pops both words and falls through with its gas by hand and no
            // depth step ("Skipping JUMPI to invalid destination", :1572-1579)
            ++executed;
            if (kind == K_JUMP) { status = ST_VMEXC; aux = EXC_BADJUMP; break; }
            if (gfent[pc] & 2u) fent = pc + 1u;     // _new_node_state on the fall-through
            sp -= 2u; ++pc; gmin += 10u; gmax += 10u;
            continue;
        }

        if (kind == K_LOG && any_sym && !tl && sp >= max(req, npop)) {
            // LOG0..4 with a symbolic operand (log_, instructions.py:1710-1723): a state
            // mutation (WriteProtection in a static call), then the words are popped and
            // nothing else happens; the table gas, then the OOG check
            const uint64_t ngmin = gmin + (d.x & 0xffffu), ngmax = gmax + (d.x >> 16);
            ++executed;
            if (flags & LANE_STATIC) { status = ST_VMEXC; aux = EXC_WRITEPROT; break; }
            if (ngmin >= glim) { status = ST_VMEXC; aux = EXC_OOG; break; }
            sp -= npop; ++pc; gmin = ngmin; gmax = ngmax;
            continue;
        }

        if (op == 0x3eu && any_sym && !tl && sp >= 3u &&
            (!sym_tag(S, N, lane, sp - 1u) || sym_never_const(S, N, lane, sym_tag(S, N, lane, sp - 1u))) &&
            (!sym_tag(S, N, lane, sp - 2u) || sym_never_const(S, N, lane, sym_tag(S, N, lane, sp - 2u))) &&
            (!sym_tag(S, N, lane, sp - 3u) || sym_never_const(S, N, lane, sym_tag(S, N, lane, sp - 3u)))) {
            // RETURNDATACOPY with a symbolic memory offset, return offset or size
            // (returndatacopy_, instructions.py:1314-1343): the three words are popped
            // and nothing is copied; the table gas, then the OOG check
            const uint64_t ngmin = gmin + (d.x & 0xffffu), ngmax = gmax + (d.x >> 16);
            ++executed;
            if (ngmin >= glim) { status = ST_VMEXC; aux = EXC_OOG; break; }
            sp -= 3u; ++pc; gmin = ngmin; gmax = ngmax;
            continue;
        }

        if (any_sym && (!tl || !tact) && (kind == K_RETURN || (kind == K_REVERT)) && sp >= 2u &&
            !(creation && kind == K_RETURN)) {
            // ---- RETURN / REVERT with a symbolic offset or length (instructions.py:
            // 1858-1934): the transaction ends; the return data are fresh
            // "return_data" bytes or a slice at symbolic keys, left to the host
            // (MG_RET_SYMBOLIC).  RETURN of a concrete length runs mem_extend, which
            // returns on a symbolic start, then check_gas_usage_limit; a symbolic
            // length skips both.  The lane stays at the instruction's start.  A taint
            // lane ends here too when its modules have no device action on the opcode.
            const uint32_t tlen = sym_tag(S, N, lane, sp - 2u);
            ++executed;
            if (kind == K_RETURN && !tlen && gmin >= glim) { status = ST_VMEXC; aux = EXC_OOG; break; }
            L.ret_offset[lane] = 0u; L.ret_len[lane] = MG_RET_SYMBOLIC;
            status = kind == K_RETURN ? ST_RETURN : ST_REVERT; aux = 0u;
            break;
        }

        if ((any_sym || env_sym || cd_sym) && !stack_op && sp >= max(req, npop)) {
            // ---- symbolic semantics: one arena node (or a concrete result) ----
            const U256 a = sp >= 1u ? V.stack(sp - 1u) : u_zero();
            const U256 b = sp >= 2u ? V.stack(sp - 2u) : u_zero();
            const uint32_t ta = sp >= 1u && nin >= 1u ? sym_tag(S, N, lane, sp - 1u) : 0u;
            const uint32_t tb = sp >= 2u && nin >= 2u ? sym_tag(S, N, lane, sp - 2u) : 0u;
            uint32_t lnn = nn, lnc = nc, rtag = 0u;
            U256 rval = u_zero();
            bool esc = false, arena_full = false, fork = false;
            uint32_t ya = 0u, yb = 0u;
            uint32_t exp_rec = 0xffffffffu;         // EXP: where its MG_REC_SYMEXP record goes
            if (kind == K_JUMPI) {
                if (ta) esc = true;                 // symbolic jump target
                else fork = true;                   // symbolic condition: the host forks
            } else if (op == 0x0au && !env_sym && !cd_sym) {
                // EXP with a symbolic operand (instructions.py:624-638): Power(base,
                // exponent), the uninterpreted function, and the manager's condition
                // on it appended to the path (the host replays the record in order)
                const uint32_t rec_at = L.rec_len[lane];
                if (tl || !L.rec_cap || (uint64_t)rec_at + MG_REC_HEADER + 1u > L.rec_cap ||
                    sym_width(S, N, lane, ta) == 1u || sym_width(S, N, lane, tb) == 1u)
                    esc = true;                     // Bool operands, taint lanes: the host
                else if (!sym_ref(S, N, lane, ta, a, lnc, ya) || !sym_ref(S, N, lane, tb, b, lnc, yb) ||
                         !sym_node_push(S, N, lane, SYM_BIN | (256u << 8), ya, yb, op, lnn, rtag))
                    arena_full = true;
                else
                    exp_rec = rec_at;
            } else if (op == 0x37u || kind == K_SHA3 || !(sym_bin_ok(op) || op == 0x15u || op == 0x19u ||
                                                          env_sym || cd_sym)) {
                esc = true;
            } else if (env_sym) {
                if (!sym_node_push(S, N, lane, SYM_ENV | (256u << 8), 0u, 0u, envw, lnn, rtag)) arena_full = true;
            } else if (op == 0x36u) {
                if (!sym_node_push(S, N, lane, SYM_CDSIZE | (256u << 8), 0u, 0u, 0u, lnn, rtag)) arena_full = true;
            } else if (op == 0x35u) {
                if (!sym_ref(S, N, lane, ta, a, lnc, ya) ||
                    !sym_node_push(S, N, lane, SYM_CDLOAD | (256u << 8), ya, 0u, 0u, lnn, rtag))
                    arena_full = true;
            } else if (op == 0x15u || op == 0x19u) {
                if (op == 0x19u && sym_width(S, N, lane, ta) == 1u) esc = true;   // 2^256-1 - Bool
                else if (!sym_ref(S, N, lane, ta, a, lnc, ya) ||
                         !sym_node_push(S, N, lane, SYM_UN | (256u << 8), ya, 0u, op, lnn, rtag))
                    arena_full = true;
            } else {
                // binary: the reference's quirks first (a concrete zero divisor gives
                // 0, a concrete BYTE index past the word gives 0, instructions.py:427-581)
                const bool zero_div = (op >= 0x04u && op <= 0x07u) && !tb && u_iszero(b);
                if (op == 0x1au && ta) esc = true;                       // symbolic BYTE index
                else if (op == 0x18u && (sym_width(S, N, lane, ta) == 1u || sym_width(S, N, lane, tb) == 1u))
                    esc = true;                                          // Bool ^ ...
                else if (zero_div || (op == 0x1au && !(u_fits32(a) && a.w[0] < 32u))) rval = u_zero();
                else if (op == 0x14u && ta && tb && sym_same(S.node, S.cval, N, lane, ta - 1u, tb - 1u))
                    rval = u_small(1u);     // x == x: the expression layer folds it (expr._fold), If(True, 1, 0)
                else if (!sym_ref(S, N, lane, ta, a, lnc, ya) || !sym_ref(S, N, lane, tb, b, lnc, yb) ||
                         !sym_node_push(S, N, lane, SYM_BIN | ((sym_is_cmp(op) ? 1u : 256u) << 8), ya, yb, op,
                                        lnn, rtag))
                    arena_full = true;
            }
            // StateTransition: table gas after the mutator, OOG, then the push
            const uint32_t nsp = sp - npop;
            const uint64_t ngmin = gmin + (d.x & 0xffffu), ngmax = gmax + (d.x >> 16);
            uint32_t stop = ST_RUNNING, sx = 0u;
            if (esc) { stop = ST_ESCAPE; sx = op | (ESC_SYMBOLIC << 8); }
            else if (fork) { stop = ST_FORK; sx = op; }
            else if (arena_full) { stop = ST_ESCAPE; sx = op | (ESC_ARENA << 8); }
            else if (pushes && nsp + 1u > STACK_LIMIT) { stop = ST_VMEXC; sx = EXC_OVERFLOW; }
            else if (pushes && nsp + 1u > L.stack_cap) { stop = ST_ESCAPE; sx = op | (ESC_STACK << 8); }
            else if (ngmin >= glim) { stop = ST_VMEXC; sx = EXC_OOG; }
            if (stop != ST_RUNNING) {
                if (rec_pre) L.rec_len[lane] = rec_save;   // the instruction did not run
                // a VmException counts as an executed step, as in k_lane_step
                if (stop != ST_ESCAPE && stop != ST_FORK) ++executed;
                status = stop; aux = sx; break;
            }
            if (tl)
                t_commit(T, N, lane, op, kind, tact, sp, nsp + 1u, nin, pushes, cd_sym, a, b, tb != 0u, pre_bit,
                         post_bit, nobj, tsink, ttf);
            if (exp_rec != 0xffffffffu) {
                uint32_t at = rec_head(L, lane, exp_rec, MG_REC_SYMEXP, 0u, L.steps[lane] + executed, u_zero());
                L.rec[(size_t)at * N + lane] = rtag - 1u;
                L.rec_len[lane] = at + 1u;
            }
            V.set_stack(nsp, rval);
            sym_set_tag(S, N, lane, nsp, rtag);
            sp = nsp + 1u; ++pc; gmin = ngmin; gmax = ngmax; nn = lnn; nc = lnc;
            if (pre_bit) { ++natoms; if (tact & T_YCLASS) tym |= pre_bit; }
            ++executed;
            continue;
        }

        // ---- concrete semantics (kernel 1's general handler); tags follow the words ----
        uint32_t t_in0 = 0u, t_in1 = 0u;
        if (symlane) {
            if (kind == K_DUP && sp >= nin) t_in0 = sym_tag(S, N, lane, sp - nin);
            if (kind == K_SWAP && sp >= nin) { t_in0 = sym_tag(S, N, lane, sp - 1u); t_in1 = sym_tag(S, N, lane, sp - nin); }
        }
        LaneRegs R{sp >= 1u ? V.stack(sp - 1u) : u_zero(), sp >= 2u ? V.stack(sp - 2u) : u_zero(), gmin, gmax,
                   pc, sp, msize, depth, n_sha3, n_exp, 0u, 0u, executed, fent};
        const U256 pa = R.T0, pb = R.T1;
        const uint32_t sp0 = sp;
        slow_step(R, E, uy, d.x);
        n_sha3 = R.n_sha3; n_exp = R.n_exp;
        if (R.stop != ST_RUNNING) {
            if (rec_pre) {
                // the mutator's own record (EXP) was not published either; drop ours
                L.rec_len[lane] = rec_save;
            }
            // halts and VmExceptions count as executed steps (k_lane_step: only an
            // escape leaves the instruction unexecuted)
            if (R.stop != ST_ESCAPE) ++executed;
            status = R.stop; aux = R.sx; break;
        }
        if (symlane && (lflags & LANE_MEMTAG) && (kind == K_CDCOPY || kind == K_CODECOPY)) {
            // the bytes a copy wrote are concrete now (CODECOPY stops at the end of
            // the code: the bytes after it keep what they held, symbolic or not)
            const U256 c = V.stack(sp0 - 3u);
            uint32_t n = 0u;
            if (kind == K_CDCOPY) n = u_iszero(c) ? 0u : c.w[0];
            else if (u_fits32(pb) && pb.w[0] < C.n_bytes) n = min(C.n_bytes - pb.w[0], c.w[0]);
            for (uint32_t j = 0; j < n; ++j) set_mtag(S, N, lane, pa.w[0] + j, 0u);
        }
        // the stack in memory is the truth here (no register window): write back
        // only the words the instruction changed -- the new top of a push or a
        // SWAP, and the second word of SWAP1 (SWAPn wrote its deep slot itself)
        if (R.sp >= 1u && (pushes || kind == K_SWAP)) V.set_stack(R.sp - 1u, R.T0);
        if (R.sp >= 2u && op == 0x90u) V.set_stack(R.sp - 2u, R.T1);
        if (symlane) {
            if (kind == K_DUP) sym_set_tag(S, N, lane, R.sp - 1u, t_in0);
            else if (kind == K_SWAP) { sym_set_tag(S, N, lane, sp - 1u, t_in1); sym_set_tag(S, N, lane, sp - nin, t_in0); }
            else if (pushes) sym_set_tag(S, N, lane, R.sp - 1u, 0u);
        }
        if (tl) {
            t_commit(T, N, lane, op, kind, tact, sp0, R.sp, nin, pushes, false, pa, pb, false, pre_bit, post_bit,
                     nobj, tsink, ttf);
            if (post_bit) {
                const uint32_t at = L.rec_len[lane];
                // the post hooks run before manage_cfg: the name before this instruction
                rec_annot(L, lane, at, natoms + (pre_bit ? 1u : 0u), L.steps[lane] + executed, R.T0,
                          R.sp >= 2u ? R.T1 : u_zero(), pc, op | 0x100u, fent);
                L.rec_len[lane] = at + TREC_WORDS;
            }
            if (pre_bit) { ++natoms; if (tact & T_YCLASS) tym |= pre_bit; }
            if (post_bit) { ++natoms; if (tact & T_YCLASS) tym |= post_bit; }
        }
        pc = R.pc; sp = R.sp; msize = R.msize; depth = R.depth; gmin = R.gmin; gmax = R.gmax; fent = R.fent;
        ++executed;
    }
    if (prof && executed != pexec) atomicAdd(&prof[pop], 1ull);

    L.pc[lane] = pc; L.sp[lane] = sp; L.msize[lane] = msize; L.depth[lane] = depth;
    L.gas_min[lane] = gmin; L.gas_max[lane] = gmax;
    L.status[lane] = status; L.aux[lane] = aux;
    L.fent[lane] = fent;
    if (hook_ack && executed > 0u) lflags &= ~LANE_HOOK_ACK;
    if (lflags != flags) L.flags[lane] = lflags;
    L.steps[lane] += executed;
    if (loop_on) L.trace_len[lane] = tlen;
    if (n_sha3) L.sha3_count[lane] += n_sha3;
    if (n_exp) L.exp_count[lane] += n_exp;
    if (symlane) { S.n_nodes[lane] = nn; S.n_consts[lane] = nc; }
    if (tl) {
        T.n_obj[lane] = nobj; T.n_atoms[lane] = natoms; T.tflags[lane] = ttf;
        T.sink[lane] = tsink; T.ymask[lane] = tym;
    }
    if (ctr) {
        DevCounters *c = ctr + lane / lanes_pb;
        atomicAdd(&c->lane_steps, (unsigned long long)executed);
        if (status != ST_RUNNING) {
            atomicSub(&c->running, 1u);
            if (status == ST_HOOK) atomicAdd(&c->hooked, 1u);
            else if (status == ST_ESCAPE || status == ST_FORK) atomicAdd(&c->escaped, 1u);
            else atomicAdd(&c->halted, 1u);
        }
    }
}
