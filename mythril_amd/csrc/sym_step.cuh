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

__global__ __launch_bounds__(256) void k_sym_step(DevLanes L, DevSym S, const DevCode *__restrict__ codes,
                                                  const uint8_t *__restrict__ a8,
                                                  const uint32_t *__restrict__ a32,
                                                  uint64_t m0, uint64_t m1, uint64_t m2, uint64_t m3,
                                                  uint32_t max_steps, uint32_t max_depth, uint32_t horizon,
                                                  DevCounters *__restrict__ ctr, uint32_t lanes_pb) {
    __shared__ uint32_t s_kc[(256u / 64u) * KC_WAVE];
    if ((threadIdx.x & 63u) < 2u) s_kc[(threadIdx.x >> 6) * KC_WAVE + KC_E * 24u + (threadIdx.x & 63u)] = 0u;
    __syncthreads();
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= L.n || L.status[lane] != ST_RUNNING) return;
    const uint32_t flags = L.flags[lane];
    if (!(flags & LANE_SYMBOLIC)) return;
    const size_t N = L.N;
    const DevCode C = codes[L.code_id[lane]];
    const uint8_t *__restrict__ gops = a8 + C.op_off;
    uint32_t pc = L.pc[lane], sp = L.sp[lane], msize = L.msize[lane], depth = L.depth[lane];
    uint64_t gmin = L.gas_min[lane], gmax = L.gas_max[lane];
    const uint64_t txlim = L.gas_limit[lane];
    const uint64_t glim = txlim < MSTATE_GAS_LIMIT + 1ull ? txlim : MSTATE_GAS_LIMIT + 1ull;
    uint32_t nn = S.n_nodes[lane], nc = S.n_consts[lane];
    const bool hook_ack = (flags & LANE_HOOK_ACK) != 0u;
    const bool creation = (flags & LANE_CREATION) != 0u;
    uint32_t lane_max = (flags & LANE_STEP1) ? min(max_steps, 1u) : max_steps;
    if (horizon) {
        const uint32_t s0 = L.steps[lane];
        lane_max = min(lane_max, horizon > s0 ? horizon - s0 : 0u);
    }
    uint32_t status = ST_RUNNING, aux = 0u, executed = 0u, n_sha3 = 0u, n_exp = 0u;
    const LaneView V{L, lane, nullptr, 0u, threadIdx.x, 256u, nullptr, 0u};
    const StepEnv E{&L, C, a8, a32, nullptr, nullptr, nullptr, nullptr, nullptr,
                    s_kc + (threadIdx.x >> 6) * KC_WAVE, txlim, glim, lane, threadIdx.x, 256u, 0u, flags,
                    0u, 0u, 0u, 0u, 0u};

    for (;;) {
        // the checks svm.execute_state makes before an instruction (svm.py:369-402)
        if (max_depth != 0u && depth >= max_depth) { status = ST_DEPTH; break; }
        if (pc >= C.n_instr) { status = ST_END; break; }
        const uint32_t op = gops[pc];
        const uint2 d = kDec[op];
        const uint32_t kind = (d.y >> 9) & 31u;
        const uint64_t hm = op < 64u ? m0 : op < 128u ? m1 : op < 192u ? m2 : m3;
        if (((hm >> (op & 63u)) & 1ull) && !(hook_ack && executed == 0u)) { status = ST_HOOK; aux = op; break; }
        if (executed >= lane_max) break;
        const uint32_t uy = op | (d.y << 8) | pd_flags(op, d.y, 0u);
        if ((uy & PD_SPECIAL) || (creation && (uy & PD_CREATION))) {
            status = ST_ESCAPE; aux = op | (ESC_OPCODE << 8); break;
        }
        const uint32_t req = d.y & 15u, npop = (d.y >> 4) & 15u;
        const bool pushes = ((d.y >> 8) & 1u) != 0u;
        uint32_t nin = npop;                        // stack words the instruction reads
        if (kind == K_DUP) nin = op - 0x7fu;
        else if (kind == K_SWAP) nin = op - 0x8fu + 1u;
        bool any_sym = false;
        for (uint32_t k = 0; k < nin && k < sp; ++k) any_sym |= sym_tag(S, N, lane, sp - 1u - k) != 0u;
        const uint32_t envw = sym_env_word(op);
        const bool env_sym = envw < 5u && ((flags >> (LANE_SYMENV_SHIFT + envw)) & 1u);
        const bool cd_sym = (flags & LANE_SYMCD) && (op == 0x35u || op == 0x36u || op == 0x37u);
        const bool stack_op = kind == K_DUP || kind == K_SWAP || kind == K_POP;

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
            if (kind == K_JUMPI) {
                if (ta) esc = true;                 // symbolic jump target
                else fork = true;                   // symbolic condition: the host forks
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
                else if (!sym_ref(S, N, lane, ta, a, lnc, ya) || !sym_ref(S, N, lane, tb, b, lnc, yb) ||
                         !sym_node_push(S, N, lane, SYM_BIN | ((sym_is_cmp(op) ? 1u : 256u) << 8), ya, yb, op,
                                        lnn, rtag))
                    arena_full = true;
            }
            if (esc) { status = ST_ESCAPE; aux = op | (ESC_SYMBOLIC << 8); break; }
            if (fork) { status = ST_FORK; aux = op; break; }
            if (arena_full) { status = ST_ESCAPE; aux = op | (ESC_ARENA << 8); break; }
            // StateTransition: table gas after the mutator, OOG, then the push
            const uint32_t nsp = sp - npop;
            if (pushes && nsp + 1u > STACK_LIMIT) { status = ST_VMEXC; aux = EXC_OVERFLOW; break; }
            if (pushes && nsp + 1u > L.stack_cap) { status = ST_ESCAPE; aux = op | (ESC_STACK << 8); break; }
            const uint64_t ngmin = gmin + (d.x & 0xffffu), ngmax = gmax + (d.x >> 16);
            if (ngmin >= glim) { status = ST_VMEXC; aux = EXC_OOG; break; }
            V.set_stack(nsp, rval);
            sym_set_tag(S, N, lane, nsp, rtag);
            sp = nsp + 1u; ++pc; gmin = ngmin; gmax = ngmax; nn = lnn; nc = lnc;
            ++executed;
            continue;
        }

        // ---- concrete semantics (kernel 1's general handler); tags follow the words ----
        uint32_t t_in0 = 0u, t_in1 = 0u;
        if (kind == K_DUP && sp >= nin) t_in0 = sym_tag(S, N, lane, sp - nin);
        if (kind == K_SWAP && sp >= nin) { t_in0 = sym_tag(S, N, lane, sp - 1u); t_in1 = sym_tag(S, N, lane, sp - nin); }
        LaneRegs R{sp >= 1u ? V.stack(sp - 1u) : u_zero(), sp >= 2u ? V.stack(sp - 2u) : u_zero(), gmin, gmax,
                   pc, sp, msize, depth, n_sha3, n_exp, 0u, 0u, executed};
        slow_step(R, E, uy, d.x);
        n_sha3 = R.n_sha3; n_exp = R.n_exp;
        if (R.stop != ST_RUNNING) { status = R.stop; aux = R.sx; break; }
        if (R.sp >= 1u) V.set_stack(R.sp - 1u, R.T0);
        if (R.sp >= 2u) V.set_stack(R.sp - 2u, R.T1);
        if (kind == K_DUP) sym_set_tag(S, N, lane, R.sp - 1u, t_in0);
        else if (kind == K_SWAP) { sym_set_tag(S, N, lane, sp - 1u, t_in1); sym_set_tag(S, N, lane, sp - nin, t_in0); }
        else if (pushes) sym_set_tag(S, N, lane, R.sp - 1u, 0u);
        pc = R.pc; sp = R.sp; msize = R.msize; depth = R.depth; gmin = R.gmin; gmax = R.gmax;
        ++executed;
    }

    L.pc[lane] = pc; L.sp[lane] = sp; L.msize[lane] = msize; L.depth[lane] = depth;
    L.gas_min[lane] = gmin; L.gas_max[lane] = gmax;
    L.status[lane] = status; L.aux[lane] = aux;
    if (hook_ack && executed > 0u) L.flags[lane] = flags & ~LANE_HOOK_ACK;
    L.steps[lane] += executed;
    if (n_sha3) L.sha3_count[lane] += n_sha3;
    if (n_exp) L.exp_count[lane] += n_exp;
    S.n_nodes[lane] = nn; S.n_consts[lane] = nc;
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
