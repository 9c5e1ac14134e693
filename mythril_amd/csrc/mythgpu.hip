// mythgpu.hip — libmythgpu.so: C-ABI, context, code tables and lane batches for
// the MI355X batched LASER core.  See include/mythgpu.h for the contract.
//
// One translation unit: the device kernels are included from lane_step.cuh
// (kernel 1, concrete lane stepper) and bv_eval.cuh (kernel 2, constraint
// prefilter).  Pure HIP runtime, no torch, no dual code paths.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mythgpu.h"
#include <cstdlib>
#include <new>
#include "bv_eval.cuh"
#include "lane_step.cuh"
#include "sym_step.cuh"
#include "cc.h"

// ------------------------------------------------------------------ context
struct mg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    // codes
    std::vector<DevCode> codes;
    std::vector<uint8_t> a8;
    std::vector<uint32_t> a32;
    uint32_t cov_total = 0;
    DevCode *d_codes = nullptr;
    uint8_t *d_a8 = nullptr;
    uint32_t *d_a32 = nullptr;
    uint8_t *d_cov = nullptr;
    size_t cap_codes = 0, cap_a8 = 0, cap_a32 = 0, cap_cov = 0;
    // lanes
    mg_batch_cfg cfg{};
    bool have_lanes = false, uploaded = false, init_fresh = false;
    uint32_t loop_bound = 0;             // mg_set_loop_bound (0: BoundedLoops off)
    uint32_t lpw = 64;                   // kernel-1 lanes per wave (MG_LANES_PER_WAVE: 64, 32, 16)
    std::vector<uint8_t> code_used;      // codes uploaded into the current batch (LDS plan)
    DevLanes L{};
    DevSym S{};                          // symbolic planes (mg_sym_alloc), freed with the lanes
    DevTaint T{};                        // taint planes (mg_taint_alloc), freed with the lanes
    uint32_t *d_tprog = nullptr;         // [256] taint action words (mg_taint_program)
    uint8_t *d_tforce = nullptr;         // per code instruction (coverage layout): host-run hooks
    size_t cap_tforce = 0;
    std::vector<void *> lane_allocs;
    // resident initial image for mg_lanes_reset
    uint32_t *i_pc = nullptr, *i_depth = nullptr, *i_status = nullptr, *i_aux = nullptr,
             *i_steps = nullptr, *i_storage_count = nullptr;
    uint64_t *i_gas_min = nullptr, *i_gas_max = nullptr;
    uint4 *i_storage = nullptr;
    // staging for upload/download (lane-major)
    void *d_stage = nullptr;
    size_t stage_bytes = 0;
    // pinned host side of the batched transfers (XferPlan): one DMA per phase
    uint8_t *h_xfer = nullptr;
    size_t h_xfer_bytes = 0;
    DevCounters *d_ctr = nullptr;        // [blocks] per-block statistics of the last launch
    uint32_t ctr_cap = 0;
    std::vector<DevCounters> h_ctr;
    // mg_run_batches: per-batch statistics slots and per-launch events
    DevCounters *d_ctr_multi = nullptr;
    size_t ctr_multi_cap = 0;            // slots
    std::vector<void *> retired;          // outgrown buffers, freed by mg_close
    // pinned host copy of the multi-batch statistics slots (a pageable D2H copy
    // is staged through a bounce buffer: ~0.1 ms for 20 C2 batches' slots)
    DevCounters *h_ctr_pin = nullptr;
    size_t h_ctr_pin_cap = 0;
    std::vector<void *> retired_host;
    std::vector<hipEvent_t> ev_batch;
    // kernel 2
    BvState bv{};
};

static int set_err(mg_ctx *ctx, int code, const char *fmt, ...) {
    if (ctx) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}
#define HIPX(ctx, call)                                                                      \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err((ctx), MG_EDEVICE, "%s failed: %s (%s:%d)", #call,               \
                           hipGetErrorString(e_), __FILE__, __LINE__);                      \
    } while (0)

// ------------------------------------------------------------- opcode table
// support/opcodes.py:16-144: gas (min, max) and STACK[0] (svm precheck count,
// with the table's own values: ADDMOD 2, EXTCODESIZE 0, SSTORE 1, DUP/SWAP 0).
static void build_optable(OpInfo t[256]) {
    std::memset(t, 0, sizeof(OpInfo) * 256);
    auto op = [&](int b, uint32_t req, uint32_t g0, uint32_t g1) { t[b] = OpInfo{g0, g1, req, 1u}; };
    op(0x00, 0, 0, 0);
    const uint32_t arith_gas[12] = {0, 3, 5, 3, 5, 5, 5, 5, 8, 8, 10, 5};
    for (int b = 0x01; b <= 0x0b; ++b) op(b, b == 0x09 ? 3 : 2, arith_gas[b], b == 0x0a ? 340 : arith_gas[b]);
    for (int b = 0x10; b <= 0x1d; ++b) op(b, (b == 0x15 || b == 0x19) ? 1 : 2, 3, 3);
    op(0x20, 2, 30, 30 + 6 * 8);
    const struct { int b; uint32_t req, g0, g1; } env[] = {
        {0x30, 0, 2, 2}, {0x31, 1, 700, 700}, {0x32, 0, 2, 2}, {0x33, 0, 2, 2}, {0x34, 0, 2, 2},
        {0x35, 1, 3, 3}, {0x36, 0, 2, 2}, {0x37, 3, 2, 2 + 3 * 768}, {0x38, 0, 2, 2},
        {0x39, 3, 2, 2 + 3 * 768}, {0x3a, 0, 2, 2}, {0x3b, 0, 700, 700},
        {0x3c, 4, 700, 700 + 3 * 768}, {0x3d, 0, 2, 2}, {0x3e, 3, 3, 3}, {0x3f, 1, 700, 700},
        {0x40, 1, 20, 20}, {0x50, 1, 2, 2}, {0x51, 1, 3, 96}, {0x52, 2, 3, 98}, {0x53, 2, 3, 98},
        {0x54, 1, 800, 800}, {0x55, 1, 5000, 25000}, {0x56, 1, 8, 8}, {0x57, 2, 10, 10},
        {0x58, 0, 2, 2}, {0x59, 0, 2, 2}, {0x5a, 0, 2, 2}, {0x5b, 0, 1, 1}, {0x5c, 0, 2, 2},
        {0x5d, 0, 5, 5}, {0x5e, 1, 10, 10}, {0xf0, 3, 32000, 32000}, {0xf5, 4, 32000, 32000},
        {0xf1, 7, 700, 34700}, {0xf2, 7, 700, 34700}, {0xf3, 2, 0, 0}, {0xf4, 6, 700, 34700},
        {0xfa, 6, 700, 34700}, {0xfd, 2, 0, 0}, {0xfe, 0, 0, 0}, {0xff, 1, 5000, 30000}};
    for (const auto &e : env) op(e.b, e.req, e.g0, e.g1);
    for (int b = 0x41; b <= 0x48; ++b) op(b, 0, 2, 2);
    for (int b = 0x60; b <= 0x9f; ++b) op(b, 0, 3, 3);   // PUSH1..32, DUP1..16, SWAP1..16
    for (int k = 0; k <= 4; ++k) op(0xa0 + k, k + 2, 375 * (k + 1), 375 * (k + 1) + 8 * 32);
}

// Opcodes that need host semantics on a concrete lane (SURVEY Appendix A #12,
// instructions.py:906-931, 1150-1435, 1699-1708, 1998-2543): symbolic block
// values, the balances array, other accounts' code, calls, creates, subroutines.
static void build_escape(uint64_t m[4]) {
    const int esc[] = {0x31, 0x3b, 0x3c, 0x3f, 0x40, 0x41, 0x42, 0x43, 0x44, 0x46, 0x47, 0x48,
                       0x5a, 0x5d, 0x5e, 0xf0, 0xf1, 0xf2, 0xf4, 0xf5, 0xfa, 0xff};
    m[0] = m[1] = m[2] = m[3] = 0;
    for (int b : esc) m[b >> 6] |= 1ull << (b & 63);
}

// Per-byte decode entry of kernel 1 (lane_step.cuh kDec): gas, precheck count,
// words popped by the mutator, whether it pushes, and the handler kind.
static void build_decode(uint2 d[256]) {
    OpInfo t[256];
    build_optable(t);
    uint64_t esc[4];
    build_escape(esc);
    for (int b = 0; b < 256; ++b) {
        uint32_t kind = K_INVALID, npop = 0, push = 0;
        if (t[b].valid && ((esc[b >> 6] >> (b & 63)) & 1ull)) kind = K_ESCAPE;
        else if (!t[b].valid || b == 0xfe) kind = K_INVALID;
        else if (b == 0x00) kind = K_STOP;
        else if ((b >= 0x01 && b <= 0x0b) || (b >= 0x10 && b <= 0x1d)) {
            kind = K_ALU; push = 1;
            npop = (b == 0x08 || b == 0x09) ? 3 : (b == 0x15 || b == 0x19) ? 1 : 2;
        } else if (b >= 0x60 && b <= 0x7f) { kind = K_PUSH; push = 1; }
        else if (b >= 0x80 && b <= 0x8f) { kind = K_DUP; push = 1; }
        else if (b >= 0x90 && b <= 0x9f) kind = K_SWAP;
        else if (b >= 0xa0 && b <= 0xa4) { kind = K_LOG; npop = 2 + (b - 0xa0); }
        else switch (b) {
            case 0x20: kind = K_SHA3; npop = 2; push = 1; break;
            case 0x30: case 0x32: case 0x33: case 0x34: case 0x36: case 0x38: case 0x3a:
            case 0x3d: case 0x45: case 0x58: case 0x59: kind = K_ENV; push = 1; break;
            case 0x35: kind = K_CDLOAD; npop = 1; push = 1; break;
            case 0x37: kind = K_CDCOPY; npop = 3; break;
            case 0x39: kind = K_CODECOPY; npop = 3; break;
            case 0x3e: kind = K_RDCOPY; npop = 3; break;
            case 0x50: kind = K_POP; npop = 1; break;
            case 0x51: kind = K_MLOAD; npop = 1; push = 1; break;
            case 0x52: kind = K_MSTORE; npop = 2; break;
            case 0x53: kind = K_MSTORE8; npop = 2; break;
            case 0x54: kind = K_SLOAD; npop = 1; push = 1; break;
            case 0x55: kind = K_SSTORE; npop = 2; break;
            case 0x56: kind = K_JUMP; npop = 1; break;
            case 0x57: kind = K_JUMPI; npop = 2; break;
            case 0x5b: kind = K_JUMPDEST; break;
            case 0x5c: kind = K_BEGINSUB; break;
            case 0xf3: kind = K_RETURN; npop = 2; break;
            case 0xfd: kind = K_REVERT; npop = 2; break;
            default: kind = K_ESCAPE; break;
        }
        d[b].x = t[b].gmin | (t[b].gmax << 16);
        d[b].y = t[b].req | (npop << 4) | (push << 8) | (kind << 9);
    }
}

extern "C" int mg_abi_version(void) { return (int)MG_ABI_VERSION; }

extern "C" int mg_opcode_info(uint32_t byte, uint32_t *gmin, uint32_t *gmax, uint32_t *req) {
    static OpInfo t[256];
    static bool ready = false;
    if (!ready) { build_optable(t); ready = true; }
    if (byte > 255 || !t[byte].valid) return -1;
    if (gmin) *gmin = t[byte].gmin;
    if (gmax) *gmax = t[byte].gmax;
    if (req) *req = t[byte].req;
    return 0;
}

extern "C" int mg_open(int device, mg_ctx **out) {
    if (!out) return MG_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MG_EDEVICE;
    if (device < 0 || device >= ndev) return MG_EINVAL;
    mg_ctx *ctx = new mg_ctx();
    ctx->device = device;
    int rc = MG_OK;
    do {
        if (hipSetDevice(device) != hipSuccess) { rc = MG_EDEVICE; break; }
        if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) { rc = MG_EDEVICE; break; }
        if (hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) { rc = MG_EDEVICE; break; }
        uint2 dec[256];
        build_decode(dec);
        if (hipMemcpyToSymbol(HIP_SYMBOL(kDec), dec, sizeof dec) != hipSuccess) { rc = MG_EDEVICE; break; }
        const char *lpw = getenv("MG_LANES_PER_WAVE");
        if (lpw && lpw[0]) {
            const long v = strtol(lpw, nullptr, 10);
            if (v != 64 && v != 32 && v != 16) { rc = MG_EINVAL; break; }
            ctx->lpw = (uint32_t)v;
        }
    } while (0);
    if (rc != MG_OK) { mg_close(ctx); return rc; }
    *out = ctx;
    return MG_OK;
}

static void free_lanes(mg_ctx *ctx) {
    for (void *p : ctx->lane_allocs) hipFree(p);
    ctx->lane_allocs.clear();
    ctx->have_lanes = ctx->uploaded = false;
    ctx->L = DevLanes{};
    ctx->S = DevSym{};
    ctx->T = DevTaint{};
    ctx->d_ctr = nullptr;
}

extern "C" void mg_close(mg_ctx *ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    free_lanes(ctx);
    bv_free(ctx->bv);
    hipFree(ctx->d_codes); hipFree(ctx->d_a8); hipFree(ctx->d_a32); hipFree(ctx->d_cov);
    hipFree(ctx->d_stage);
    hipFree(ctx->d_tprog);
    hipFree(ctx->d_tforce);
    if (ctx->ev0) hipEventDestroy(ctx->ev0);
    if (ctx->ev1) hipEventDestroy(ctx->ev1);
    for (hipEvent_t e : ctx->ev_batch) hipEventDestroy(e);
    hipFree(ctx->d_ctr_multi);
    for (void *p : ctx->retired) hipFree(p);
    if (ctx->h_ctr_pin) hipHostFree(ctx->h_ctr_pin);
    for (void *p : ctx->retired_host) hipHostFree(p);
    if (ctx->h_xfer) hipHostFree(ctx->h_xfer);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
}

extern "C" const char *mg_last_error(mg_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// -------------------------------------------------------------------- code
// Python's repr of a bytes object: asm.py:107-123 tests `"bzzr" in str(bytes[-43:])`.
static std::string py_bytes_repr(const uint8_t *p, size_t n) {
    bool sq = false, dq = false;
    for (size_t i = 0; i < n; ++i) { sq |= p[i] == '\''; dq |= p[i] == '"'; }
    const char q = (sq && !dq) ? '"' : '\'';
    static const char hx[] = "0123456789abcdef";
    std::string s = "b";
    s += q;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t c = p[i];
        if (c == (uint8_t)q || c == '\\') { s += '\\'; s += (char)c; }
        else if (c == '\t') s += "\\t";
        else if (c == '\n') s += "\\n";
        else if (c == '\r') s += "\\r";
        else if (c < 32 || c >= 127) { s += "\\x"; s += hx[c >> 4]; s += hx[c & 15]; }
        else s += (char)c;
    }
    s += q;
    return s;
}

template <class T>
static int ensure_dev(mg_ctx *ctx, T *&ptr, size_t &cap, size_t need) {
    if (need <= cap && ptr) return MG_OK;
    size_t ncap = std::max(need, cap * 2 + 64);
    T *p = nullptr;
    if (hipMalloc(&p, ncap * sizeof(T)) != hipSuccess) return set_err(ctx, MG_ENOMEM, "hipMalloc code arena");
    hipFree(ptr);
    ptr = p;
    cap = ncap;
    return MG_OK;
}

// Disassembly (asm.py:99-148) + get_instruction_index (util.py:45-59) tables.
extern "C" int mg_load_code(mg_ctx *ctx, const uint8_t *code, size_t n, uint32_t *code_id) {
    if (!ctx || (!code && n) || !code_id) return set_err(ctx, MG_EINVAL, "mg_load_code: bad args");
    if (n > (1u << 30)) return set_err(ctx, MG_EINVAL, "mg_load_code: code too large");
    OpInfo t[256];
    build_optable(t);
    size_t length = n;
    const size_t tail = std::min<size_t>(n, 43);
    if (py_bytes_repr(code + n - tail, tail).find("bzzr") != std::string::npos)
        length = n >= 43 ? n - 43 : 0;
    std::vector<uint8_t> ops;
    std::vector<uint32_t> addrs, push;
    // the argument as Disassembly's instruction_list holds it ("0x" + the bytes
    // present in the code, asm.py:136-142: a PUSH at the end is truncated, not
    // padded) as an integer, for the dispatcher table below; UINT64_MAX when it
    // has no byte (int("0x", 16) fails) or cannot be an address
    std::vector<uint64_t> argv;
    size_t a = 0;
    while (a < length) {
        const uint8_t b = code[a];
        uint32_t pv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        uint64_t av = UINT64_MAX;
        addrs.push_back((uint32_t)a);
        if (!t[b].valid) {
            ops.push_back(0xfe);
        } else {
            ops.push_back(b);
            if (b >= 0x60 && b <= 0x7f) {
                const size_t np = b - 0x5f;
                // argument from the FULL bytecode, right-padded with zeros (instructions.py:316)
                for (size_t i = 0; i < np; ++i) {
                    const uint8_t v = (a + 1 + i < n) ? code[a + 1 + i] : 0;
                    const size_t bit = 8 * (np - 1 - i);
                    pv[bit / 32] |= (uint32_t)v << (bit % 32);
                }
                const size_t present = std::min(np, n - (a + 1));
                if (present > 0) {
                    av = 0;
                    for (size_t i = 0; i < present && av != UINT64_MAX; ++i)
                        av = av >> 40 ? UINT64_MAX : (av << 8) | code[a + 1 + i];
                }
                a += np;
            }
        }
        argv.push_back(av);
        push.insert(push.end(), pv, pv + 8);
        a += 1;
    }
    // Dispatcher entries (Disassembly.assign_bytecode, disassembly.py:36-56):
    // every PUSH1..PUSH4 followed by EQ (asm.find_op_code_sequence, asm.py:66-94)
    // whose next instruction is a PUSH names an entry point = that PUSH's argument
    // (get_function_info, disassembly.py:106-114); address_to_function_name is keyed
    // by it, and _new_node_state (svm.py:617-637) switches the function name when a
    // JUMP / JUMPI lands on the instruction at exactly that address; address 0
    // switches it to "fallback".  fent[i]: bit 0 for index i, bit 1 for i + 1.
    std::vector<uint8_t> fent(ops.size() + 1, 0);
    if (!ops.empty()) fent[0] = 1;
    for (size_t i = 0; i + 2 < ops.size(); ++i) {
        if (ops[i] < 0x60 || ops[i] > 0x63 || ops[i + 1] != 0x14) continue;
        if (ops[i + 2] < 0x60 || ops[i + 2] > 0x7f || argv[i + 2] > 0xffffffffull) continue;
        const auto it = std::lower_bound(addrs.begin(), addrs.end(), (uint32_t)argv[i + 2]);
        if (it != addrs.end() && *it == (uint32_t)argv[i + 2]) fent[it - addrs.begin()] = 1;
    }
    for (size_t i = 0; i < ops.size(); ++i) fent[i] = (uint8_t)((fent[i] & 1u) | ((fent[i + 1] & 1u) << 1));
    DevCode dc{};
    dc.n_instr = (uint32_t)ops.size();
    dc.n_bytes = (uint32_t)n;
    dc.n_jres = dc.n_instr ? addrs.back() + 1u : 0u;
    // arena8: ops, bytes
    dc.op_off = (uint32_t)ctx->a8.size();
    ctx->a8.insert(ctx->a8.end(), ops.begin(), ops.end());
    dc.bytes_off = (uint32_t)ctx->a8.size();
    ctx->a8.insert(ctx->a8.end(), code, code + n);
    dc.fent_off = (uint32_t)ctx->a8.size();
    ctx->a8.insert(ctx->a8.end(), fent.begin(), fent.begin() + ops.size());
    while (ctx->a8.size() % 16) ctx->a8.push_back(0);
    // arena32: push (32-byte aligned), addr, jres
    while (ctx->a32.size() % 8) ctx->a32.push_back(0);
    dc.push_off = (uint32_t)ctx->a32.size();
    ctx->a32.insert(ctx->a32.end(), push.begin(), push.end());
    dc.addr_off = (uint32_t)ctx->a32.size();
    ctx->a32.insert(ctx->a32.end(), addrs.begin(), addrs.end());
    dc.jres_off = (uint32_t)ctx->a32.size();
    {
        size_t k = 0;
        for (uint32_t tgt = 0; tgt < dc.n_jres; ++tgt) {
            while (k < addrs.size() && addrs[k] < tgt) ++k;
            ctx->a32.push_back(k < addrs.size() ? (uint32_t)k : MG_JRES_NONE);
        }
    }
    // straight-line runs (kernel 1's block path): from every instruction, the
    // run of simple opcodes (PUSH/DUP/SWAP/POP/JUMPDEST/fast ALU) that follows,
    // at most RUN_MAX long, optionally ended by one JUMP or JUMPI, with the stack
    // depth it needs, the growth it peaks at and the table gas of its simple
    // part (jumps add their 8 / 10 by hand), so a lane can check once and
    // execute the run without per-instruction checks (lane_step.cuh).
    // rx = len | need << 8 | peak << 16 | jump kind << 24 (1 JUMP, 2 JUMPI).
    {
        const size_t ni = ops.size();
        std::vector<uint32_t> rx(ni + 1, 0u), ry(ni + 1, 0u);
        std::vector<int> need(ni + 1, 0), peak(ni + 1, 0), len(ni + 1, 0), jk(ni + 1, 0);
        std::vector<uint32_t> g0(ni + 1, 0u), g1(ni + 1, 0u);
        for (size_t i = ni; i-- > 0;) {
            const uint32_t b = ops[i];
            int req = -1, d = 0;
            if (b >= 0x60 && b <= 0x7f) { req = 0; d = 1; }
            else if (b >= 0x80 && b <= 0x8f) { req = (int)(b - 0x7f); d = 1; }
            else if (b >= 0x90 && b <= 0x9f) { req = (int)(b - 0x8e); d = 0; }
            else if (b == 0x50) { req = 1; d = -1; }
            else if (b == 0x5b) { req = 0; d = 0; }
            else if (b == 0x15 || b == 0x19) { req = 1; d = 0; }
            else if (b <= 0x03 && b >= 0x01) { req = 2; d = -1; }
            else if (b == 0x0b || (b >= 0x10 && b <= 0x1d)) { req = 2; d = -1; }
            if (b == 0x56 || b == 0x57) {               // a jump ends the run it closes
                len[i] = 1;
                need[i] = b == 0x56 ? 1 : 2;
                peak[i] = 0;
                jk[i] = b == 0x56 ? 1 : 2;
                g0[i] = g1[i] = 0u;
                rx[i] = 1u | ((uint32_t)need[i] << 8) | ((uint32_t)jk[i] << 24);
                ry[i] = 0u;
                continue;
            }
            if (req < 0) continue;                      // not simple: runs end here
            const bool cont = len[i + 1] > 0 && len[i + 1] < RUN_MAX;
            len[i] = 1 + (cont ? len[i + 1] : 0);
            need[i] = std::max(req, (cont ? need[i + 1] : 0) - d);
            peak[i] = std::max(0, d + (cont ? peak[i + 1] : 0));
            jk[i] = cont ? jk[i + 1] : 0;
            g0[i] = t[b].gmin + (cont ? g0[i + 1] : 0u);
            g1[i] = t[b].gmax + (cont ? g1[i + 1] : 0u);
            rx[i] = (uint32_t)len[i] | ((uint32_t)need[i] << 8) | ((uint32_t)peak[i] << 16) |
                    ((uint32_t)jk[i] << 24);
            ry[i] = g0[i] | (g1[i] << 16);
        }
        dc.run_off = (uint32_t)ctx->a32.size();
        for (size_t i = 0; i < ni; ++i) { ctx->a32.push_back(rx[i]); ctx->a32.push_back(ry[i]); }
    }
    dc.cov_off = ctx->cov_total;
    ctx->cov_total += dc.n_instr + 1u;
    ctx->codes.push_back(dc);
    // re-upload arenas (small)
    int rc;
    if ((rc = ensure_dev(ctx, ctx->d_codes, ctx->cap_codes, ctx->codes.size()))) return rc;
    if ((rc = ensure_dev(ctx, ctx->d_a8, ctx->cap_a8, ctx->a8.size() + 16))) return rc;
    if ((rc = ensure_dev(ctx, ctx->d_a32, ctx->cap_a32, ctx->a32.size() + 16))) return rc;
    const size_t old_cov = ctx->cap_cov;
    uint8_t *old_cov_ptr = ctx->d_cov;
    if (ctx->cov_total > ctx->cap_cov) {
        uint8_t *p = nullptr;
        const size_t ncap = std::max<size_t>(ctx->cov_total, 2 * ctx->cap_cov + 256);
        if (hipMalloc(&p, ncap) != hipSuccess) return set_err(ctx, MG_ENOMEM, "hipMalloc coverage");
        HIPX(ctx, hipMemsetAsync(p, 0, ncap, ctx->stream));
        if (old_cov_ptr) HIPX(ctx, hipMemcpyAsync(p, old_cov_ptr, old_cov, hipMemcpyDeviceToDevice, ctx->stream));
        HIPX(ctx, hipStreamSynchronize(ctx->stream));
        hipFree(old_cov_ptr);
        ctx->d_cov = p;
        ctx->cap_cov = ncap;
    }
    HIPX(ctx, hipMemcpyAsync(ctx->d_codes, ctx->codes.data(), ctx->codes.size() * sizeof(DevCode),
                             hipMemcpyHostToDevice, ctx->stream));
    HIPX(ctx, hipMemcpyAsync(ctx->d_a8, ctx->a8.data(), ctx->a8.size(), hipMemcpyHostToDevice, ctx->stream));
    HIPX(ctx, hipMemcpyAsync(ctx->d_a32, ctx->a32.data(), ctx->a32.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    *code_id = (uint32_t)(ctx->codes.size() - 1);
    return MG_OK;
}

extern "C" int mg_code_info(mg_ctx *ctx, uint32_t code_id, uint32_t *n_instr) {
    if (!ctx || code_id >= ctx->codes.size()) return set_err(ctx, MG_ENOCODE, "unknown code_id %u", code_id);
    if (n_instr) *n_instr = ctx->codes[code_id].n_instr;
    return MG_OK;
}

extern "C" int mg_code_fentries(mg_ctx *ctx, uint32_t code_id, uint8_t *out, uint32_t n) {
    if (!ctx || code_id >= ctx->codes.size()) return set_err(ctx, MG_ENOCODE, "unknown code_id %u", code_id);
    const DevCode &c = ctx->codes[code_id];
    if (!out || n != c.n_instr) return set_err(ctx, MG_EINVAL, "mg_code_fentries: need %u bytes", c.n_instr);
    std::memcpy(out, ctx->a8.data() + c.fent_off, n);
    return MG_OK;
}

extern "C" int mg_code_table(mg_ctx *ctx, uint32_t code_id, uint8_t *ops, uint32_t *addrs, uint32_t n) {
    if (!ctx || code_id >= ctx->codes.size()) return set_err(ctx, MG_ENOCODE, "unknown code_id %u", code_id);
    const DevCode &c = ctx->codes[code_id];
    if (!ops || !addrs || n != c.n_instr) return set_err(ctx, MG_EINVAL, "mg_code_table: need %u entries", c.n_instr);
    std::memcpy(ops, ctx->a8.data() + c.op_off, n);
    std::memcpy(addrs, ctx->a32.data() + c.addr_off, (size_t)n * 4);
    return MG_OK;
}

// ------------------------------------------------------------------- lanes
template <class T>
static int lane_alloc(mg_ctx *ctx, T *&p, size_t count) {
    void *q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess)
        return set_err(ctx, MG_ENOMEM, "hipMalloc %zu bytes for lanes", count * sizeof(T));
    ctx->lane_allocs.push_back(q);
    p = (T *)q;
    return MG_OK;
}

extern "C" int mg_lanes_alloc(mg_ctx *ctx, const mg_batch_cfg *cfg) {
    if (!ctx || !cfg) return MG_EINVAL;
    if (cfg->n_lanes == 0 || cfg->stack_cap == 0 || cfg->stack_cap > MG_STACK_LIMIT ||
        cfg->mem_cap % 32 || cfg->calldata_cap % 4 || cfg->storage_cap == 0)
        return set_err(ctx, MG_EINVAL, "mg_lanes_alloc: bad batch configuration");
    HIPX(ctx, hipSetDevice(ctx->device));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    free_lanes(ctx);
    ctx->code_used.assign(ctx->codes.size(), 0);
    ctx->cfg = *cfg;
    DevLanes &L = ctx->L;
    L.n = cfg->n_lanes;
    L.N = (cfg->n_lanes + 63u) & ~63u;
    L.stack_cap = cfg->stack_cap; L.mem_cap = cfg->mem_cap;
    L.calldata_cap = std::max<uint32_t>(cfg->calldata_cap, 4u); L.storage_cap = cfg->storage_cap;
    const size_t N = L.N;
    int rc = 0;
    uint32_t **u32s[] = {&L.code_id, &L.pc, &L.sp, &L.msize, &L.depth, &L.status, &L.aux, &L.steps,
                         &L.flags, &L.calldata_len, &L.storage_count, &L.ret_offset, &L.ret_len,
                         &L.sha3_count, &L.exp_count, &L.fent, &ctx->i_pc, &ctx->i_depth, &ctx->i_status,
                         &ctx->i_aux, &ctx->i_steps, &ctx->i_storage_count};
    for (auto pp : u32s)
        if ((rc = lane_alloc(ctx, *pp, N))) return rc;
    uint64_t **u64s[] = {&L.gas_min, &L.gas_max, &L.gas_limit, &ctx->i_gas_min, &ctx->i_gas_max};
    for (auto pp : u64s)
        if ((rc = lane_alloc(ctx, *pp, N))) return rc;
    if ((rc = lane_alloc(ctx, L.stack, (size_t)L.stack_cap * N * 2))) return rc;
    if ((rc = lane_alloc(ctx, L.mem, (size_t)(L.mem_cap / 4) * N))) return rc;
    if ((rc = lane_alloc(ctx, L.calldata, (size_t)(L.calldata_cap / 4) * N))) return rc;
    if ((rc = lane_alloc(ctx, L.env, (size_t)MG_ENV_WORDS * N * 2))) return rc;
    if ((rc = lane_alloc(ctx, L.storage, (size_t)L.storage_cap * N * 4))) return rc;
    if ((rc = lane_alloc(ctx, ctx->i_storage, (size_t)L.storage_cap * N * 4))) return rc;
    L.trace_cap = cfg->trace_cap;
    if ((rc = lane_alloc(ctx, L.trace_len, N))) return rc;
    if (L.trace_cap && (rc = lane_alloc(ctx, L.trace, (size_t)L.trace_cap * N))) return rc;
    HIPX(ctx, hipMemsetAsync(L.trace_len, 0, N * 4, ctx->stream));
    // per-block launch statistics (summed on the host)
    ctx->ctr_cap = (uint32_t)(N / (LANE_BLOCK / 4u) + 1);   // lpw >= 16
    if ((rc = lane_alloc(ctx, ctx->d_ctr, (size_t)ctx->ctr_cap))) return rc;
    L.rec_cap = cfg->rec_cap;
    if ((rc = lane_alloc(ctx, L.rec_len, N))) return rc;
    if (L.rec_cap && (rc = lane_alloc(ctx, L.rec, (size_t)L.rec_cap * N))) return rc;
    HIPX(ctx, hipMemsetAsync(L.rec_len, 0, N * 4, ctx->stream));
    // no lane runs before upload
    HIPX(ctx, hipMemsetAsync(L.status, 0xff, N * 4, ctx->stream));
    HIPX(ctx, hipMemsetAsync(L.sha3_count, 0, N * 4, ctx->stream));
    HIPX(ctx, hipMemsetAsync(L.exp_count, 0, N * 4, ctx->stream));
    HIPX(ctx, hipMemsetAsync(L.fent, 0xff, N * 4, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    ctx->have_lanes = true;
    ctx->cfg.calldata_cap = L.calldata_cap;
    return MG_OK;
}

// ---- lane transfers: stage (lane-major rows) <-> device (unit-major, lanes interleaved)
// A field of U units x W dwords per lane lives on the device as
// dst[(u * N + lane) * W + k]; the host stage holds each lane's row contiguously,
// src[(lane * U + u) * W + k].  One block moves a tile of 64 lanes x 64 dwords
// (64 / W units) through LDS, so both the row reads and the unit-major writes
// are contiguous runs (a per-element kernel writes one side at stride N * W).
// Byte fields (memory, calldata) are W = 1 with each dword byte-swapped: the
// stage holds bytes, the device big-endian dwords.  W is a power of two <= 64.
#define XT_LANES 64u
#define XT_COLS 64u
template <bool BSWAP>
__global__ __launch_bounds__(256) void k_xfer_scatter(const uint32_t *__restrict__ src, uint32_t n, uint32_t U,
                                                     uint32_t lgW, uint32_t *__restrict__ dst, uint32_t N,
                                                     uint32_t first) {
    __shared__ uint32_t tile[XT_LANES][XT_COLS + 1];
    const uint32_t W = 1u << lgW, TU = XT_COLS >> lgW;
    const uint32_t l0 = blockIdx.x * XT_LANES, u0 = blockIdx.y * TU;
    const uint32_t nl = min(XT_LANES, n - l0), nu = min(TU, U - u0), cols = nu << lgW;
    const size_t row = (size_t)U << lgW;
    for (uint32_t i = threadIdx.x; i < XT_LANES * XT_COLS; i += blockDim.x) {
        const uint32_t l = i / XT_COLS, c = i % XT_COLS;
        if (l < nl && c < cols) {
            uint32_t v = src[(size_t)(l0 + l) * row + ((size_t)u0 << lgW) + c];
            tile[l][c] = BSWAP ? __builtin_bswap32(v) : v;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < XT_LANES * XT_COLS; i += blockDim.x) {
        const uint32_t uo = i / (XT_LANES * W), rem = i % (XT_LANES * W);
        const uint32_t l = rem >> lgW, k = rem & (W - 1u);
        if (uo < nu && l < nl)
            dst[(((size_t)(u0 + uo) * N + first + l0 + l) << lgW) + k] = tile[l][(uo << lgW) + k];
    }
}
template <bool BSWAP>
__global__ __launch_bounds__(256) void k_xfer_gather(const uint32_t *__restrict__ src, uint32_t n, uint32_t U,
                                                    uint32_t lgW, uint32_t *__restrict__ dst, uint32_t N,
                                                    uint32_t first) {
    __shared__ uint32_t tile[XT_LANES][XT_COLS + 1];
    const uint32_t W = 1u << lgW, TU = XT_COLS >> lgW;
    const uint32_t l0 = blockIdx.x * XT_LANES, u0 = blockIdx.y * TU;
    const uint32_t nl = min(XT_LANES, n - l0), nu = min(TU, U - u0), cols = nu << lgW;
    const size_t row = (size_t)U << lgW;
    for (uint32_t i = threadIdx.x; i < XT_LANES * XT_COLS; i += blockDim.x) {
        const uint32_t uo = i / (XT_LANES * W), rem = i % (XT_LANES * W);
        const uint32_t l = rem >> lgW, k = rem & (W - 1u);
        if (uo < nu && l < nl) {
            const uint32_t v = src[(((size_t)(u0 + uo) * N + first + l0 + l) << lgW) + k];
            tile[l][(uo << lgW) + k] = BSWAP ? __builtin_bswap32(v) : v;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < XT_LANES * XT_COLS; i += blockDim.x) {
        const uint32_t l = i / XT_COLS, c = i % XT_COLS;
        if (l < nl && c < cols) dst[(size_t)(l0 + l) * row + ((size_t)u0 << lgW) + c] = tile[l][c];
    }
}
static uint32_t lg2(uint32_t w) { uint32_t r = 0; while ((1u << r) < w) ++r; return r; }
static dim3 xfer_grid(uint32_t n, uint32_t U, uint32_t W) {
    return dim3((n + XT_LANES - 1) / XT_LANES, (U + (XT_COLS / W) - 1) / (XT_COLS / W));
}
// restore the working state from the resident initial image
__global__ void k_reset(DevLanes L, DevResetImage R) {
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= L.n) return;
    reset_lane(L, R, lane);
}

static int ensure_stage(mg_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->stage_bytes) return MG_OK;
    hipFree(ctx->d_stage);
    ctx->d_stage = nullptr;
    ctx->stage_bytes = 0;
    if (hipMalloc(&ctx->d_stage, bytes) != hipSuccess) return set_err(ctx, MG_ENOMEM, "hipMalloc staging %zu", bytes);
    ctx->stage_bytes = bytes;
    return MG_OK;
}

static unsigned blocks_for(size_t work, unsigned bs = 256) { return (unsigned)((work + bs - 1) / bs); }

// ---- batched transfers ---------------------------------------------------------
// One host<->device transfer of many lane fields.  Download: every field is
// gathered (lane-major) into the device stage, ONE DMA copies the stage into a
// pinned host buffer, ONE stream synchronisation, then the host copies the
// rows into the caller's arrays.  Upload: the rows are packed into the pinned
// buffer, ONE DMA, then scatter kernels / device copies (the caller syncs once).
// The per-field form it replaced (pageable copy + synchronisation per field,
// now ab/xfer_legacy.diff) cost ~2.5 ms per LaserEVM launch (profiles/r03/hostprof).
struct XferPlan {
    enum Kind { SCALAR, UNITS, BYTES };
    struct Item {
        Kind kind;
        void *host;             // caller's array (lane-major rows)
        void *dev, *dev2;       // device field (dev2: a second destination on upload)
        size_t elem;            // SCALAR: bytes per lane
        uint32_t Uh, W, Uc;     // UNITS: host row of Uh units x W dwords, Uc units copied; BYTES: W = 0, Uh/Uc dwords
        size_t off, len;        // in the stage
    };
    std::vector<Item> items;
    bool bad = false;           // a field the transfer kernels cannot move
    size_t total = 0;
    uint32_t n = 0, first = 0;
    XferPlan(uint32_t n_, uint32_t first_) : n(n_), first(first_) {}
    void add(Item it) {
        if (!it.host) return;
        if (it.kind == SCALAR) it.len = (size_t)n * it.elem;
        else {
            it.Uc = std::min(it.Uc, it.Uh);
            if (it.Uc == 0 || n == 0) return;
            it.len = (size_t)n * it.Uc * (it.kind == UNITS ? it.W : 1u) * 4u;
        }
        it.off = total;
        total += (it.len + 15u) & ~(size_t)15u;
        items.push_back(it);
    }
    void scalar(void *host, void *dev, size_t elem, void *dev2 = nullptr) {
        add(Item{SCALAR, host, dev, dev2, elem, 0, 0, 0, 0, 0});
    }
    void units(void *host, uint32_t Uh, uint32_t W, void *dev, uint32_t Uc = 0xffffffffu, void *dev2 = nullptr) {
        // the transpose kernels take W as a power of two up to a tile row
        if (W == 0 || (W & (W - 1u)) || W > XT_COLS) { bad = true; return; }
        if (Uh) add(Item{UNITS, host, dev, dev2, 0, Uh, W, Uc, 0, 0});
    }
    void bytes(void *host, uint32_t bytes_h, void *dev, uint32_t Dc = 0xffffffffu) {
        if (bytes_h) add(Item{BYTES, host, dev, nullptr, 0, bytes_h / 4u, 0, Dc, 0, 0});
    }
};

static uint32_t max_of(const uint32_t *v, uint32_t n) {
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; ++i) m = std::max(m, v[i]);
    return m;
}

static int ensure_hxfer(mg_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->h_xfer_bytes) return MG_OK;
    // geometric growth: a slowly growing transfer reallocates pinned memory
    // (milliseconds per hipHostFree + hipHostMalloc) only O(log n) times
    const size_t cap = std::max<size_t>(bytes, 2 * ctx->h_xfer_bytes + (1u << 20));
    if (ctx->h_xfer) hipHostFree(ctx->h_xfer);
    ctx->h_xfer = nullptr;
    ctx->h_xfer_bytes = 0;
    if (hipHostMalloc((void **)&ctx->h_xfer, cap, hipHostMallocDefault) != hipSuccess)
        return set_err(ctx, MG_ENOMEM, "hipHostMalloc transfer buffer %zu", cap);
    ctx->h_xfer_bytes = cap;
    return MG_OK;
}

// a row of `row_c` bytes out of every `row_h`-byte host row: one copy when whole
static void rows_copy(uint8_t *dst, size_t dst_row, const uint8_t *src, size_t src_row, size_t row, uint32_t n) {
    if (dst_row == row && src_row == row) { std::memcpy(dst, src, row * n); return; }
    for (uint32_t i = 0; i < n; ++i) std::memcpy(dst + i * dst_row, src + i * src_row, row);
}

static int xfer_down(mg_ctx *ctx, const XferPlan &x) {
    if (x.bad) return set_err(ctx, MG_EINVAL, "lane transfer: unit width not a power of two <= 64");
    if (x.items.empty()) return MG_OK;
    int rc;
    if ((rc = ensure_stage(ctx, x.total)) || (rc = ensure_hxfer(ctx, x.total))) return rc;
    uint8_t *ds = (uint8_t *)ctx->d_stage;
    const uint32_t N = ctx->L.N;
    for (const auto &it : x.items) {
        if (it.kind == XferPlan::SCALAR) {
            HIPX(ctx, hipMemcpyAsync(ds + it.off, (const uint8_t *)it.dev + (size_t)x.first * it.elem, it.len,
                                     hipMemcpyDeviceToDevice, ctx->stream));
        } else if (it.kind == XferPlan::UNITS) {
            hipLaunchKernelGGL(k_xfer_gather<false>, xfer_grid(x.n, it.Uc, it.W), dim3(256), 0, ctx->stream,
                               (const uint32_t *)it.dev, x.n, it.Uc, lg2(it.W), (uint32_t *)(ds + it.off), N,
                               x.first);
        } else {
            hipLaunchKernelGGL(k_xfer_gather<true>, xfer_grid(x.n, it.Uc, 1), dim3(256), 0, ctx->stream,
                               (const uint32_t *)it.dev, x.n, it.Uc, 0u, (uint32_t *)(ds + it.off), N, x.first);
        }
    }
    HIPX(ctx, hipGetLastError());
    HIPX(ctx, hipMemcpyAsync(ctx->h_xfer, ds, x.total, hipMemcpyDeviceToHost, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    for (const auto &it : x.items) {
        const uint8_t *src = ctx->h_xfer + it.off;
        if (it.kind == XferPlan::SCALAR) {
            std::memcpy(it.host, src, it.len);
        } else {
            const size_t unit = it.kind == XferPlan::UNITS ? (size_t)it.W * 4u : 4u;
            rows_copy((uint8_t *)it.host, it.Uh * unit, src, it.Uc * unit, it.Uc * unit, x.n);
        }
    }
    return MG_OK;
}

// enqueues the upload; the caller synchronises the stream (h_xfer is reused)
static int xfer_up(mg_ctx *ctx, const XferPlan &x) {
    if (x.bad) return set_err(ctx, MG_EINVAL, "lane transfer: unit width not a power of two <= 64");
    if (x.items.empty()) return MG_OK;
    int rc;
    if ((rc = ensure_stage(ctx, x.total)) || (rc = ensure_hxfer(ctx, x.total))) return rc;
    for (const auto &it : x.items) {
        uint8_t *dst = ctx->h_xfer + it.off;
        if (it.kind == XferPlan::SCALAR) {
            std::memcpy(dst, it.host, it.len);
        } else {
            const size_t unit = it.kind == XferPlan::UNITS ? (size_t)it.W * 4u : 4u;
            rows_copy(dst, it.Uc * unit, (const uint8_t *)it.host, it.Uh * unit, it.Uc * unit, x.n);
        }
    }
    uint8_t *ds = (uint8_t *)ctx->d_stage;
    HIPX(ctx, hipMemcpyAsync(ds, ctx->h_xfer, x.total, hipMemcpyHostToDevice, ctx->stream));
    const uint32_t N = ctx->L.N;
    for (const auto &it : x.items) {
        for (void *dev : {it.dev, it.dev2}) {
            if (!dev) continue;
            if (it.kind == XferPlan::SCALAR) {
                HIPX(ctx, hipMemcpyAsync((uint8_t *)dev + (size_t)x.first * it.elem, ds + it.off, it.len,
                                         hipMemcpyDeviceToDevice, ctx->stream));
            } else if (it.kind == XferPlan::UNITS) {
                hipLaunchKernelGGL(k_xfer_scatter<false>, xfer_grid(x.n, it.Uc, it.W), dim3(256), 0, ctx->stream,
                                   (const uint32_t *)(ds + it.off), x.n, it.Uc, lg2(it.W), (uint32_t *)dev, N,
                                   x.first);
            } else {
                hipLaunchKernelGGL(k_xfer_scatter<true>, xfer_grid(x.n, it.Uc, 1), dim3(256), 0, ctx->stream,
                                   (const uint32_t *)(ds + it.off), x.n, it.Uc, 0u, (uint32_t *)dev, N, x.first);
            }
        }
    }
    HIPX(ctx, hipGetLastError());
    return MG_OK;
}

static int check_host_shape(mg_ctx *ctx, const mg_lane_soa *h, uint32_t first, uint32_t n) {
    if (!ctx->have_lanes) return set_err(ctx, MG_ESTATE, "mg_lanes_alloc first");
    if (!h || h->n != n || first + (uint64_t)n > ctx->L.n)
        return set_err(ctx, MG_EINVAL, "lane range [%u,%u) outside batch of %u (host n=%u)", first,
                       first + n, ctx->L.n, h ? h->n : 0);
    if (h->stack_cap > ctx->L.stack_cap || h->mem_cap > ctx->L.mem_cap || h->mem_cap % 4 ||
        h->calldata_cap > ctx->L.calldata_cap || h->calldata_cap % 4 || h->storage_cap > ctx->L.storage_cap ||
        h->trace_cap > ctx->L.trace_cap || h->rec_cap > ctx->L.rec_cap)
        return set_err(ctx, MG_EINVAL, "host image capacities exceed the batch configuration");
    return MG_OK;
}

static int lanes_upload(mg_ctx *ctx, const mg_lane_soa *h, uint32_t first, uint32_t n, bool live);

extern "C" int mg_lanes_upload(mg_ctx *ctx, const mg_lane_soa *h, uint32_t first, uint32_t n) {
    return lanes_upload(ctx, h, first, n, false);
}

extern "C" int mg_lanes_upload_live(mg_ctx *ctx, const mg_lane_soa *h, uint32_t first, uint32_t n) {
    return lanes_upload(ctx, h, first, n, true);
}

static int lanes_upload(mg_ctx *ctx, const mg_lane_soa *h, uint32_t first, uint32_t n, bool live) {
    if (!ctx) return MG_EINVAL;
    int rc;
    if ((rc = check_host_shape(ctx, h, first, n))) return rc;
    HIPX(ctx, hipSetDevice(ctx->device));
    DevLanes &L = ctx->L;
    // validate code ids and capacities on the host before any kernel sees them
    if (ctx->code_used.size() < ctx->codes.size()) ctx->code_used.resize(ctx->codes.size(), 0);
    for (uint32_t i = 0; i < n; ++i) {
        if (h->code_id[i] >= ctx->codes.size()) return set_err(ctx, MG_ENOCODE, "lane %u: unknown code_id", first + i);
        ctx->code_used[h->code_id[i]] = 1;
        if (h->sp[i] > h->stack_cap || h->msize[i] > h->mem_cap || h->msize[i] % 32 ||
            h->calldata_len[i] > h->calldata_cap || h->storage_count[i] > h->storage_cap ||
            (h->trace_cap ? h->trace_len[i] > h->trace_cap : 0u) ||
            (h->rec_cap ? h->rec_len[i] > h->rec_cap : 0u))
            return set_err(ctx, MG_EINVAL, "lane %u: state exceeds its host capacities", first + i);
    }
    bool fresh = true;
    for (uint32_t i = 0; i < n && fresh; ++i)
        fresh = h->sp[i] == 0 && h->msize[i] == 0 && (!h->trace_cap || h->trace_len[i] == 0) &&
                (!h->rec_cap || h->rec_len[i] == 0);
    const uint32_t ALL = 0xffffffffu;
    XferPlan x(n, first);
    x.scalar(h->code_id, L.code_id, 4);
    x.scalar(h->pc, L.pc, 4, ctx->i_pc);
    x.scalar(h->sp, L.sp, 4);
    x.scalar(h->msize, L.msize, 4);
    x.scalar(h->depth, L.depth, 4, ctx->i_depth);
    x.scalar(h->status, L.status, 4, ctx->i_status);
    x.scalar(h->aux, L.aux, 4, ctx->i_aux);
    x.scalar(h->steps, L.steps, 4, ctx->i_steps);
    x.scalar(h->flags, L.flags, 4);
    x.scalar(h->calldata_len, L.calldata_len, 4);
    x.scalar(h->storage_count, L.storage_count, 4, ctx->i_storage_count);
    x.scalar(h->ret_offset, L.ret_offset, 4);
    x.scalar(h->ret_len, L.ret_len, 4);
    x.scalar(h->gas_min, L.gas_min, 8, ctx->i_gas_min);
    x.scalar(h->gas_max, L.gas_max, 8, ctx->i_gas_max);
    x.scalar(h->gas_limit, L.gas_limit, 8);
    if (h->fent) x.scalar(h->fent, L.fent, 4);
    // rows below the range's largest sp / storage count / msize / trace and record
    // length: no step reads above them before writing (pushes write their slot,
    // stores and logs append, memory is zero-filled when it extends), so the rest
    // of each capacity never crosses PCIe (`live` only leaves out env and calldata)
    (void)ALL;
    x.units(h->stack, h->stack_cap, 8, L.stack, max_of(h->sp, n));
    x.units(h->env, MG_ENV_WORDS, 8, L.env);
    x.units(h->storage, h->storage_cap, 16, L.storage, max_of(h->storage_count, n), ctx->i_storage);
    x.bytes(h->memory, h->mem_cap, L.mem, (max_of(h->msize, n) + 3u) / 4u);
    x.bytes(h->calldata, h->calldata_cap, L.calldata);
    if (h->trace_cap) {
        x.scalar(h->trace_len, L.trace_len, 4);
        x.units(h->trace, h->trace_cap, 1, L.trace, max_of(h->trace_len, n));
    }
    if (h->rec_cap) {
        x.scalar(h->rec_len, L.rec_len, 4);
        x.units(h->rec, h->rec_cap, 1, L.rec, max_of(h->rec_len, n));
    }
    HIPX(ctx, hipMemsetAsync(L.sha3_count + first, 0, (size_t)n * 4, ctx->stream));
    HIPX(ctx, hipMemsetAsync(L.exp_count + first, 0, (size_t)n * 4, ctx->stream));
    if (!h->trace_cap) HIPX(ctx, hipMemsetAsync(L.trace_len + first, 0, (size_t)n * 4, ctx->stream));
    if (!h->rec_cap) HIPX(ctx, hipMemsetAsync(L.rec_len + first, 0, (size_t)n * 4, ctx->stream));
    if (!h->fent) HIPX(ctx, hipMemsetAsync(L.fent + first, 0xff, (size_t)n * 4, ctx->stream));
    if ((rc = xfer_up(ctx, x))) return rc;
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    ctx->uploaded = true;
    ctx->init_fresh = (first == 0 && n == L.n) ? fresh : (ctx->init_fresh && fresh);
    return MG_OK;
}

// ---- symbolic planes ---------------------------------------------------------
extern "C" int mg_sym_alloc(mg_ctx *ctx, uint32_t node_cap, uint32_t const_cap) {
    if (!ctx) return MG_EINVAL;
    if (!ctx->have_lanes) return set_err(ctx, MG_ESTATE, "mg_sym_alloc before mg_lanes_alloc");
    if (ctx->S.node) return set_err(ctx, MG_ESTATE, "mg_sym_alloc: already allocated for this batch");
    if (node_cap == 0u || const_cap == 0u || node_cap >= SYM_CONST || const_cap >= SYM_CONST)
        return set_err(ctx, MG_EINVAL, "mg_sym_alloc: bad capacities");
    HIPX(ctx, hipSetDevice(ctx->device));
    DevSym S{};
    S.node_cap = node_cap;
    S.const_cap = const_cap;
    const size_t N = ctx->L.N;
    auto get = [&](void **p, size_t bytes) -> int {
        if (hipMalloc(p, bytes) != hipSuccess) return set_err(ctx, MG_ENOMEM, "mg_sym_alloc: %zu bytes", bytes);
        ctx->lane_allocs.push_back(*p);
        return hipMemsetAsync(*p, 0, bytes, ctx->stream) == hipSuccess ? MG_OK : MG_EDEVICE;
    };
    int rc;
    if ((rc = get((void **)&S.stag, (size_t)ctx->L.stack_cap * N * 4))) return rc;
    if ((rc = get((void **)&S.node, (size_t)node_cap * N * 16))) return rc;
    if ((rc = get((void **)&S.cval, (size_t)const_cap * N * 32))) return rc;
    if ((rc = get((void **)&S.n_nodes, N * 4))) return rc;
    if ((rc = get((void **)&S.n_consts, N * 4))) return rc;
    if ((rc = get((void **)&S.mtag, (size_t)ctx->L.mem_cap * N * 4))) return rc;
    if ((rc = get((void **)&S.sttag, (size_t)ctx->L.storage_cap * N * 8))) return rc;
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    ctx->S = S;
    return MG_OK;
}

static int check_sym_shape(mg_ctx *ctx, const mg_sym_soa *h, uint32_t first, uint32_t n) {
    if (!ctx->S.node) return set_err(ctx, MG_ESTATE, "mg_sym_alloc first");
    if (!h || h->n != n || first + (uint64_t)n > ctx->L.n)
        return set_err(ctx, MG_EINVAL, "symbolic lane range [%u,%u) outside batch of %u", first, first + n, ctx->L.n);
    if (h->stack_cap > ctx->L.stack_cap || h->node_cap > ctx->S.node_cap || h->const_cap > ctx->S.const_cap ||
        h->mem_cap > ctx->L.mem_cap || h->storage_cap > ctx->L.storage_cap)
        return set_err(ctx, MG_EINVAL, "symbolic host image capacities exceed the allocation");
    return MG_OK;
}

extern "C" int mg_sym_upload(mg_ctx *ctx, const mg_sym_soa *h, uint32_t first, uint32_t n) {
    if (!ctx) return MG_EINVAL;
    int rc;
    if ((rc = check_sym_shape(ctx, h, first, n))) return rc;
    HIPX(ctx, hipSetDevice(ctx->device));
    for (uint32_t i = 0; i < n; ++i)
        if (h->n_nodes[i] > h->node_cap || h->n_consts[i] > h->const_cap)
            return set_err(ctx, MG_EINVAL, "lane %u: arena exceeds its host capacities", first + i);
    // the arena only grows from each lane's node / constant count and no step reads a
    // row past it: rows up to the range's largest count cross PCIe, not the capacity
    XferPlan x(n, first);
    x.scalar(h->n_nodes, ctx->S.n_nodes, 4);
    x.scalar(h->n_consts, ctx->S.n_consts, 4);
    x.units(h->stag, h->stack_cap, 1, ctx->S.stag);
    x.units(h->node, h->node_cap, 4, ctx->S.node, max_of(h->n_nodes, n));
    x.units(h->cval, h->const_cap, 8, ctx->S.cval, max_of(h->n_consts, n));
    x.units(h->mtag, h->mem_cap, 1, ctx->S.mtag);
    x.units(h->sttag, h->storage_cap, 2, ctx->S.sttag);
    if ((rc = xfer_up(ctx, x))) return rc;
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

extern "C" int mg_sym_download(mg_ctx *ctx, mg_sym_soa *h, uint32_t first, uint32_t n) {
    if (!ctx) return MG_EINVAL;
    int rc;
    if ((rc = check_sym_shape(ctx, h, first, n))) return rc;
    HIPX(ctx, hipSetDevice(ctx->device));
    // phase 1: the counts (they bound phase 2's arena rows)
    XferPlan x(n, first);
    x.scalar(h->n_nodes, ctx->S.n_nodes, 4);
    x.scalar(h->n_consts, ctx->S.n_consts, 4);
    if ((rc = xfer_down(ctx, x))) return rc;
    XferPlan y(n, first);
    y.units(h->stag, h->stack_cap, 1, ctx->S.stag);
    y.units(h->node, h->node_cap, 4, ctx->S.node, max_of(h->n_nodes, n));
    y.units(h->cval, h->const_cap, 8, ctx->S.cval, max_of(h->n_consts, n));
    y.units(h->mtag, h->mem_cap, 1, ctx->S.mtag);
    y.units(h->sttag, h->storage_cap, 2, ctx->S.sttag);
    return xfer_down(ctx, y);
}

// ---- taint planes ------------------------------------------------------------
static int ensure_tprog(mg_ctx *ctx) {
    if (ctx->d_tprog) return MG_OK;
    HIPX(ctx, hipMalloc((void **)&ctx->d_tprog, 256 * 4));
    HIPX(ctx, hipMemsetAsync(ctx->d_tprog, 0, 256 * 4, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

extern "C" int mg_taint_alloc(mg_ctx *ctx, uint32_t obj_cap) {
    if (!ctx) return MG_EINVAL;
    if (!ctx->have_lanes) return set_err(ctx, MG_ESTATE, "mg_taint_alloc before mg_lanes_alloc");
    if (ctx->T.sobj) return set_err(ctx, MG_ESTATE, "mg_taint_alloc: already allocated for this batch");
    if (obj_cap < MG_TAINT_OBJ0 + 8u || obj_cap > 65536u)
        return set_err(ctx, MG_EINVAL, "mg_taint_alloc: obj_cap %u outside [%u, 65536]", obj_cap, MG_TAINT_OBJ0 + 8u);
    HIPX(ctx, hipSetDevice(ctx->device));
    int rc;
    if ((rc = ensure_tprog(ctx))) return rc;
    DevTaint T{};
    T.obj_cap = obj_cap;
    T.prog = ctx->d_tprog;
    T.force = ctx->d_tforce;
    const size_t N = ctx->L.N;
    auto get = [&](void **p, size_t bytes) -> int {
        if (hipMalloc(p, bytes) != hipSuccess) return set_err(ctx, MG_ENOMEM, "mg_taint_alloc: %zu bytes", bytes);
        ctx->lane_allocs.push_back(*p);
        return hipMemsetAsync(*p, 0, bytes, ctx->stream) == hipSuccess ? MG_OK : MG_EDEVICE;
    };
    if ((rc = get((void **)&T.sobj, (size_t)ctx->L.stack_cap * N * 4))) return rc;
    if ((rc = get((void **)&T.omask, (size_t)obj_cap * N * 8))) return rc;
    if ((rc = get((void **)&T.oremap, (size_t)obj_cap * N * 4))) return rc;
    if ((rc = get((void **)&T.n_obj, N * 4))) return rc;
    if ((rc = get((void **)&T.n_fixed, N * 4))) return rc;
    if ((rc = get((void **)&T.n_atoms, N * 4))) return rc;
    if ((rc = get((void **)&T.tflags, N * 4))) return rc;
    if ((rc = get((void **)&T.sink, N * 8))) return rc;
    if ((rc = get((void **)&T.ymask, N * 8))) return rc;
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    ctx->T = T;
    return MG_OK;
}

extern "C" int mg_taint_program(mg_ctx *ctx, const uint32_t actions[256]) {
    if (!ctx || !actions) return MG_EINVAL;
    HIPX(ctx, hipSetDevice(ctx->device));
    for (int k = 0; k < 256; ++k) {
        const uint32_t a = actions[k];
        if (a & ~0x1ffff7fu) return set_err(ctx, MG_EINVAL, "taint action %#x of opcode %#x: unknown bits", a, k);
        if ((a & 15u) > 7u || ((a >> 8) & 15u) > 7u || ((a >> 12) & 15u) > 7u || ((a >> 16) & 15u) > 3u ||
            ((a >> 20) & 15u) > 7u)
            return set_err(ctx, MG_EINVAL, "taint action %#x of opcode %#x: operand out of range", a, k);
    }
    int rc;
    if ((rc = ensure_tprog(ctx))) return rc;
    HIPX(ctx, hipMemcpyAsync(ctx->d_tprog, actions, 256 * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

extern "C" int mg_taint_force(mg_ctx *ctx, uint32_t code_id, const uint8_t *flags, uint32_t n) {
    if (!ctx || !flags) return MG_EINVAL;
    if (code_id >= ctx->codes.size()) return set_err(ctx, MG_ENOCODE, "unknown code_id %u", code_id);
    const DevCode &c = ctx->codes[code_id];
    if (n != c.n_instr) return set_err(ctx, MG_EINVAL, "mg_taint_force: %u flags for %u instructions", n, c.n_instr);
    HIPX(ctx, hipSetDevice(ctx->device));
    if (ctx->cov_total > ctx->cap_tforce) {
        uint8_t *p = nullptr;
        const size_t ncap = std::max<size_t>(ctx->cov_total, 2 * ctx->cap_tforce + 256);
        HIPX(ctx, hipMalloc((void **)&p, ncap));
        HIPX(ctx, hipMemsetAsync(p, 0, ncap, ctx->stream));
        if (ctx->d_tforce) HIPX(ctx, hipMemcpyAsync(p, ctx->d_tforce, ctx->cap_tforce, hipMemcpyDeviceToDevice, ctx->stream));
        HIPX(ctx, hipStreamSynchronize(ctx->stream));
        hipFree(ctx->d_tforce);
        ctx->d_tforce = p;
        ctx->cap_tforce = ncap;
    }
    HIPX(ctx, hipMemcpyAsync(ctx->d_tforce + c.cov_off, flags, n, hipMemcpyHostToDevice, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    ctx->T.force = ctx->d_tforce;
    return MG_OK;
}

static int check_taint_shape(mg_ctx *ctx, const mg_taint_soa *h, uint32_t first, uint32_t n) {
    if (!ctx->T.sobj) return set_err(ctx, MG_ESTATE, "mg_taint_alloc first");
    if (!h || h->n != n || first + (uint64_t)n > ctx->L.n)
        return set_err(ctx, MG_EINVAL, "taint lane range [%u,%u) outside batch of %u", first, first + n, ctx->L.n);
    if (h->stack_cap > ctx->L.stack_cap || h->obj_cap > ctx->T.obj_cap)
        return set_err(ctx, MG_EINVAL, "taint host image capacities exceed the allocation");
    return MG_OK;
}

extern "C" int mg_taint_upload(mg_ctx *ctx, const mg_taint_soa *h, uint32_t first, uint32_t n) {
    if (!ctx) return MG_EINVAL;
    int rc;
    if ((rc = check_taint_shape(ctx, h, first, n))) return rc;
    HIPX(ctx, hipSetDevice(ctx->device));
    for (uint32_t i = 0; i < n; ++i) {
        if (h->n_obj[i] > h->obj_cap || h->n_fixed[i] < MG_TAINT_OBJ0 || h->n_fixed[i] > h->n_obj[i] ||
            h->n_atoms[i] > 64u)
            return set_err(ctx, MG_EINVAL, "lane %u: taint counts outside its capacities", first + i);
        // slots above the lane's sp may hold stale handles (never read before a push
        // writes them); every handle must index the object table
        const uint32_t *so = h->sobj + (size_t)i * h->stack_cap;
        for (uint32_t k = 0; k < h->stack_cap; ++k)
            if (so[k] >= h->obj_cap)
                return set_err(ctx, MG_EINVAL, "lane %u slot %u: handle %u past obj_cap", first + i, k, so[k]);
    }
    DevTaint &T = ctx->T;
    XferPlan x(n, first);
    x.scalar(h->n_obj, T.n_obj, 4);
    x.scalar(h->n_fixed, T.n_fixed, 4);
    x.scalar(h->n_atoms, T.n_atoms, 4);
    x.scalar(h->tflags, T.tflags, 4);
    x.scalar(h->sink, T.sink, 8);
    x.scalar(h->ymask, T.ymask, 8);
    x.units(h->sobj, h->stack_cap, 1, T.sobj);
    x.units(h->omask, h->obj_cap, 2, T.omask, max_of(h->n_obj, n));    // objects past n_obj are unread
    if ((rc = xfer_up(ctx, x))) return rc;
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

extern "C" int mg_taint_download(mg_ctx *ctx, mg_taint_soa *h, uint32_t first, uint32_t n) {
    if (!ctx) return MG_EINVAL;
    int rc;
    if ((rc = check_taint_shape(ctx, h, first, n))) return rc;
    HIPX(ctx, hipSetDevice(ctx->device));
    DevTaint &T = ctx->T;
    XferPlan x(n, first);
    x.scalar(h->n_obj, T.n_obj, 4);
    x.scalar(h->n_fixed, T.n_fixed, 4);
    x.scalar(h->n_atoms, T.n_atoms, 4);
    x.scalar(h->tflags, T.tflags, 4);
    x.scalar(h->sink, T.sink, 8);
    x.scalar(h->ymask, T.ymask, 8);
    if ((rc = xfer_down(ctx, x))) return rc;
    XferPlan y(n, first);
    y.units(h->sobj, h->stack_cap, 1, T.sobj);
    y.units(h->omask, h->obj_cap, 2, T.omask, max_of(h->n_obj, n));
    return xfer_down(ctx, y);
}


static int lanes_download(mg_ctx *ctx, mg_lane_soa *h, uint32_t first, uint32_t n, bool live);

extern "C" int mg_lanes_download(mg_ctx *ctx, mg_lane_soa *h, uint32_t first, uint32_t n) {
    return lanes_download(ctx, h, first, n, false);
}

extern "C" int mg_lanes_download_live(mg_ctx *ctx, mg_lane_soa *h, uint32_t first, uint32_t n) {
    return lanes_download(ctx, h, first, n, true);
}

static int lanes_download(mg_ctx *ctx, mg_lane_soa *h, uint32_t first, uint32_t n, bool live) {
    if (!ctx) return MG_EINVAL;
    int rc;
    if ((rc = check_host_shape(ctx, h, first, n))) return rc;
    HIPX(ctx, hipSetDevice(ctx->device));
    DevLanes &L = ctx->L;
    // phase 1: the per-lane scalars (they bound phase 2's rows)
    XferPlan x(n, first);
    x.scalar(h->code_id, L.code_id, 4);
    x.scalar(h->pc, L.pc, 4);
    x.scalar(h->sp, L.sp, 4);
    x.scalar(h->msize, L.msize, 4);
    x.scalar(h->depth, L.depth, 4);
    x.scalar(h->status, L.status, 4);
    x.scalar(h->aux, L.aux, 4);
    x.scalar(h->steps, L.steps, 4);
    x.scalar(h->flags, L.flags, 4);
    x.scalar(h->calldata_len, L.calldata_len, 4);
    x.scalar(h->storage_count, L.storage_count, 4);
    x.scalar(h->ret_offset, L.ret_offset, 4);
    x.scalar(h->ret_len, L.ret_len, 4);
    x.scalar(h->gas_min, L.gas_min, 8);
    x.scalar(h->gas_max, L.gas_max, 8);
    x.scalar(h->gas_limit, L.gas_limit, 8);
    if (h->trace_cap) x.scalar(h->trace_len, L.trace_len, 4);
    if (h->rec_cap) x.scalar(h->rec_len, L.rec_len, 4);
    if (h->fent) x.scalar(h->fent, L.fent, 4);
    if ((rc = xfer_down(ctx, x))) return rc;
    // phase 2: rows; live: only what a step can have written, below the
    // range's largest sp / storage count / msize / trace and record length
    const uint32_t ALL = 0xffffffffu;
    XferPlan y(n, first);
    y.units(h->stack, h->stack_cap, 8, L.stack, live ? max_of(h->sp, n) : ALL);
    if (!live) y.units(h->env, MG_ENV_WORDS, 8, L.env);
    y.units(h->storage, h->storage_cap, 16, L.storage, live ? max_of(h->storage_count, n) : ALL);
    y.bytes(h->memory, h->mem_cap, L.mem, live ? (max_of(h->msize, n) + 3u) / 4u : ALL);
    if (!live) y.bytes(h->calldata, h->calldata_cap, L.calldata);
    if (h->trace_cap) y.units(h->trace, h->trace_cap, 1, L.trace, live ? max_of(h->trace_len, n) : ALL);
    if (h->rec_cap) y.units(h->rec, h->rec_cap, 1, L.rec, live ? max_of(h->rec_len, n) : ALL);
    return xfer_down(ctx, y);
}

extern "C" int mg_set_loop_bound(mg_ctx *ctx, uint32_t bound) {
    if (!ctx) return MG_EINVAL;
    ctx->loop_bound = bound;
    return MG_OK;
}

static DevResetImage reset_image(const mg_ctx *ctx) {
    return DevResetImage{ctx->i_pc, ctx->i_depth, ctx->i_status, ctx->i_aux, ctx->i_steps,
                         ctx->i_storage_count, ctx->i_gas_min, ctx->i_gas_max, ctx->i_storage};
}

extern "C" int mg_lanes_reset(mg_ctx *ctx) {
    if (!ctx) return MG_EINVAL;
    if (!ctx->uploaded) return set_err(ctx, MG_ESTATE, "mg_lanes_reset before mg_lanes_upload");
    if (!ctx->init_fresh)
        return set_err(ctx, MG_ESTATE, "mg_lanes_reset needs an uploaded image with empty stacks and memory");
    hipLaunchKernelGGL(k_reset, dim3(blocks_for(ctx->L.n)), dim3(256), 0, ctx->stream, ctx->L, reset_image(ctx));
    HIPX(ctx, hipGetLastError());
    return MG_OK;
}

// LDS plan of one launch.  One block's share of the 160 KiB CU budget (64 / lpw
// blocks per CU, one wave per SIMD each) minus a margin for the static arrays
// holds the stack window (2 x 16 B per lane of the block per slot: 8 KiB at 256
// lanes, at most 16 slots) and the largest loaded code: pre-decoded entries
// (16 B per instruction + the END sentinel), coverage bytes (1 B) and the
// jump-resolve table (2 B per byte address).  When the whole code, its push
// immediates (32 B per instruction) and a 16-slot window fit, everything is
// staged (push_lds).  Otherwise the push immediates stay in the code arena
// (read at wave-uniform addresses), the window shrinks to MIN_WIN slots, and the
// code gets the rest: a prefix of the instructions and of the jump targets when
// even that is too little (lane_step.cuh decodes the remainder from HBM).
// lanes per kernel-1 workgroup: 4 waves of ctx->lpw lanes
static inline uint32_t lane_block(const mg_ctx *ctx) { return (LANE_BLOCK / 64u) * ctx->lpw; }

struct LdsPlan {
    uint32_t win, pd_cap, jr_cap, push_lds, mw32;   // mw32: memory window, 32-byte words per lane
    size_t bytes;
};

// default LDS memory window per lane (bytes, multiple of 32): Solidity's scratch
// words, free-memory pointer, zero slot and first allocation (0x00-0x9f)
#define MEMWIN_DEFAULT 160u

static LdsPlan lds_plan(const mg_ctx *ctx) {
    static const uint32_t MAX_WIN = 16u, MIN_WIN = 10u;
    // sized for the largest code the batch's lanes were uploaded with (all codes
    // when none is marked)
    uint32_t maxn = 0, maxj = 0;
    bool any = false;
    for (size_t k = 0; k < ctx->code_used.size() && k < ctx->codes.size(); ++k) any |= ctx->code_used[k] != 0;
    for (size_t k = 0; k < ctx->codes.size(); ++k) {
        if (any && (k >= ctx->code_used.size() || !ctx->code_used[k])) continue;
        maxn = std::max(maxn, ctx->codes[k].n_instr); maxj = std::max(maxj, ctx->codes[k].n_jres);
    }
    const size_t budget = 160u * 1024u / (64u / ctx->lpw) - 6144u;
    const size_t slot_bytes = 2u * lane_block(ctx) * 16u;
    const uint32_t win_cap = std::min<uint32_t>(MAX_WIN, ctx->L.stack_cap);
    LdsPlan p{};
    const uint32_t pd_full = (std::min<uint32_t>(maxn, 0xfffeu) + 1u + 15u) & ~15u;   // + END sentinel
    const uint32_t jr_full = (maxj + 15u) & ~15u;
    const size_t full = (size_t)pd_full * (16 + 32 + 1) + (size_t)jr_full * 2;
    if (maxn < 0xfffeu && full + (size_t)win_cap * slot_bytes <= budget) {
        p.pd_cap = pd_full; p.jr_cap = jr_full; p.push_lds = 1u;
    } else {
        const size_t min_win = std::min<uint32_t>(MIN_WIN, win_cap);
        const size_t avail = budget > min_win * slot_bytes ? budget - min_win * slot_bytes : 0;
        p.pd_cap = (uint32_t)std::min<size_t>(pd_full, (avail / 17u) & ~(size_t)15u);
        p.jr_cap = (uint32_t)std::min<size_t>(jr_full, ((avail - (size_t)p.pd_cap * 17u) / 2u) & ~(size_t)15u);
        p.push_lds = 0u;
    }
    // test / A/B overrides: MG_K1_PUSH=global, MG_K1_PD_CAP=n, MG_K1_JR_CAP=n (a
    // smaller staged prefix exercises the HBM-decoded remainder on small codes)
    const char *ev = getenv("MG_K1_PUSH");
    if (ev && std::string(ev) == "global") p.push_lds = 0u;
    if ((ev = getenv("MG_K1_PD_CAP")) != nullptr) {
        const uint32_t c = (uint32_t)strtoul(ev, nullptr, 10);
        if (c >= 1u && c < p.pd_cap) { p.pd_cap = c; p.push_lds = 0u; }
    }
    if ((ev = getenv("MG_K1_JR_CAP")) != nullptr) {
        const uint32_t c = (uint32_t)strtoul(ev, nullptr, 10);
        if (c < p.jr_cap) p.jr_cap = c;
    }
    const size_t code_bytes = (size_t)p.pd_cap * (16 + (p.push_lds ? 32 : 0) + 1) + (size_t)p.jr_cap * 2;
    // memory window (MG_K1_MEMWIN=bytes overrides; 0 = off): taken from the stack
    // window's share only while that keeps at least MIN_WIN slots
    uint32_t mwb = MEMWIN_DEFAULT;
    if ((ev = getenv("MG_K1_MEMWIN")) != nullptr) mwb = (uint32_t)strtoul(ev, nullptr, 10);
    mwb = std::min<uint32_t>(std::min<uint32_t>(mwb, ctx->L.mem_cap), 255u * 32u) & ~31u;
    const size_t lanes = lane_block(ctx);
    size_t left = budget > code_bytes ? budget - code_bytes : 0;
    const size_t min_stack = (size_t)std::min<uint32_t>(MIN_WIN, win_cap) * slot_bytes;
    while (mwb > 0u && (size_t)mwb * lanes + min_stack > left) mwb -= 32u;
    p.mw32 = mwb / 32u;
    left -= (size_t)mwb * lanes;
    p.win = (uint32_t)std::min<size_t>(win_cap, left / slot_bytes);
    p.bytes = (size_t)p.win * slot_bytes + (size_t)mwb * lanes + code_bytes + 16;
    return p;
}

// MG_K1_RUNS=reg: straight-line runs in the register form only (the fallback
// form; forced for the parity tests and A/B runs,
// read per launch so one process can alternate the two forms)
static uint32_t k1_flags() {
    const char *r = getenv("MG_K1_RUNS");
    return (r && std::string(r) == "reg") ? 0x100u : 0u;
}

// plan / kflags: a caller launching many batches computes the LDS plan and the
// environment switches once (getenv scans the environment: ~1-2 us a call, five
// calls per launch were most of the gap between C2 batches)
static int launch_step(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps, uint32_t max_depth,
                       DevCounters *ctr, unsigned long long *prof = nullptr, uint32_t horizon = 0,
                       const DevResetImage *reset = nullptr, const LdsPlan *plan = nullptr,
                       int64_t kflags = -1) {
    const uint64_t zero[4] = {0, 0, 0, 0};
    const uint64_t *m = hook_mask ? hook_mask : zero;
    const LdsPlan P = plan ? *plan : lds_plan(ctx);
    if (ctx->loop_bound && ctx->L.trace_cap) {
        // the loop-count hash compares 16-bit byte addresses (EVM code < 64 KiB)
        for (const DevCode &c : ctx->codes)
            if (c.n_bytes > 65536u) return set_err(ctx, MG_EINVAL, "loop bound needs codes below 64 KiB");
    }
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)k_lane_step<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024 - 6144);
        (void)hipFuncSetAttribute((const void *)k_lane_step<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024 - 6144);
        (void)hipGetLastError();   // the attribute is advisory on gfx950; never leave a sticky error
        attr_set = true;
    }
    const uint32_t loop_bound = ctx->L.trace_cap ? ctx->loop_bound : 0u;
    if (ctr && blocks_for(ctx->L.n, lane_block(ctx)) > ctx->ctr_cap)
        return set_err(ctx, MG_EINVAL, "launch of %u blocks exceeds the %u statistics slots",
                       blocks_for(ctx->L.n, lane_block(ctx)), ctx->ctr_cap);
    hipLaunchKernelGGL(loop_bound ? k_lane_step<true> : k_lane_step<false>, dim3(blocks_for(ctx->L.n, lane_block(ctx))),
                       dim3(LANE_BLOCK), P.bytes, ctx->stream, ctx->L,
                       ctx->d_codes, ctx->d_a8, ctx->d_a32, ctx->d_cov, ctx->cfg.coverage ? 1u : 0u, m[0], m[1],
                       m[2], m[3], max_steps, max_depth, ctr, prof, P.win, P.pd_cap, P.jr_cap, horizon,
                       loop_bound, reset ? *reset : DevResetImage{},
                       ctx->lpw | (kflags >= 0 ? (uint32_t)kflags : k1_flags()) | (P.push_lds ? 0x200u : 0u) |
                       (P.mw32 << 16));
    HIPX(ctx, hipGetLastError());
    // symbolic and taint lanes: the concrete stepper left them untouched (counted as running)
    // (a profiling pass counts their opcodes into the same histogram)
    if ((ctx->S.node || ctx->T.sobj) && !reset) {
        hipLaunchKernelGGL(k_sym_step, dim3(blocks_for(ctx->L.n)), dim3(256), 0, ctx->stream, ctx->L, ctx->S,
                           ctx->T, ctx->d_codes, ctx->d_a8, ctx->d_a32, m[0], m[1], m[2], m[3], max_steps, max_depth,
                           horizon, loop_bound, ctr, lane_block(ctx), prof);
        HIPX(ctx, hipGetLastError());
    }
    return MG_OK;
}

#ifdef MG_K1_CLOCKS
// diagnostic build only: the per-wave cycle bins of the last kernel-1 launch
extern "C" int mg_k1_clocks(mg_ctx *ctx, uint32_t *out, size_t n) {
    if (!ctx || !out) return MG_EINVAL;
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    HIPX(ctx, hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k1_clk), std::min<size_t>(n, 4096u * CLK_BINS) * 4u));
    return MG_OK;
}
#endif

extern "C" int mg_step(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps, uint32_t max_depth,
                       mg_step_stats *stats) {
    return mg_step_until(ctx, hook_mask, max_steps, max_depth, 0u, stats);
}

extern "C" int mg_step_until(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps, uint32_t max_depth,
                             uint32_t horizon, mg_step_stats *stats) {
    if (!ctx) return MG_EINVAL;
    if (!ctx->uploaded) return set_err(ctx, MG_ESTATE, "mg_step before mg_lanes_upload");
    HIPX(ctx, hipSetDevice(ctx->device));
    HIPX(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    int rc = launch_step(ctx, hook_mask, max_steps, max_depth, ctx->d_ctr, nullptr, horizon);
    if (rc) return rc;
    HIPX(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    const uint32_t nb = blocks_for(ctx->L.n, lane_block(ctx));
    ctx->h_ctr.resize(nb);
    HIPX(ctx, hipMemcpyAsync(ctx->h_ctr.data(), ctx->d_ctr, nb * sizeof(DevCounters), hipMemcpyDeviceToHost,
                             ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    DevCounters c{};
    for (const DevCounters &b : ctx->h_ctr) {
        c.lane_steps += b.lane_steps; c.running += b.running; c.halted += b.halted;
        c.hooked += b.hooked; c.escaped += b.escaped;
    }
    if (stats) {
        float ms = 0.f;
        HIPX(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        stats->lane_steps = c.lane_steps;
        stats->running = c.running;
        stats->halted = c.halted;
        stats->hooked = c.hooked;
        stats->escaped = c.escaped;
        stats->kernel_ms = ms;
        stats->launches = 1;
    }
    return MG_OK;
}

// Whole batches back to back on the stream: each batch re-initialises every
// lane from the resident image and steps it (one k_lane_step launch),
// with its own statistics slots and a HIP event pair around its stepping
// kernel; the host waits once, after the last batch.  This is the
// throughput form of `for i in range(n): mg_lanes_reset(); mg_step(...)`
// (no host round trip between batches).
extern "C" int mg_run_batches(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps, uint32_t max_depth,
                              uint32_t n_batches, mg_step_stats *stats) {
    if (!ctx) return MG_EINVAL;
    if (!stats || n_batches == 0u) return set_err(ctx, MG_EINVAL, "mg_run_batches needs n_batches > 0 and stats");
    if (!ctx->uploaded) return set_err(ctx, MG_ESTATE, "mg_run_batches before mg_lanes_upload");
    if (!ctx->init_fresh)
        return set_err(ctx, MG_ESTATE, "mg_run_batches needs an uploaded image with empty stacks and memory");
    HIPX(ctx, hipSetDevice(ctx->device));
    const uint32_t nb = blocks_for(ctx->L.n, lane_block(ctx));
    const size_t slots = (size_t)nb * n_batches;
    if (slots > ctx->ctr_multi_cap) {
        // grow geometrically and retire the old buffer instead of freeing it: hipFree
        // waits for the whole device, which would serialise another context's
        // stream running on the same GPU (two contexts per GPU)
        HIPX(ctx, hipStreamSynchronize(ctx->stream));
        const size_t cap = std::max(slots, std::max(2 * ctx->ctr_multi_cap, (size_t)nb * 64u));
        DevCounters *p = nullptr;
        if (hipMalloc(&p, cap * sizeof(DevCounters)) != hipSuccess)
            return set_err(ctx, MG_ENOMEM, "hipMalloc %zu statistics slots", cap);
        if (ctx->d_ctr_multi) ctx->retired.push_back(ctx->d_ctr_multi);
        ctx->d_ctr_multi = p;
        ctx->ctr_multi_cap = cap;
        DevCounters *hp = nullptr;
        if (hipHostMalloc((void **)&hp, cap * sizeof(DevCounters), hipHostMallocDefault) != hipSuccess)
            return set_err(ctx, MG_ENOMEM, "hipHostMalloc %zu statistics slots", cap);
        if (ctx->h_ctr_pin) ctx->retired_host.push_back(ctx->h_ctr_pin);
        ctx->h_ctr_pin = hp;
        ctx->h_ctr_pin_cap = cap;
    }
    // events in a block of at least 128 (64 batches): like the statistics slots,
    // created before they are needed rather than on a larger call's first use
    while (ctx->ev_batch.size() < std::max<size_t>(2u * n_batches, 128u)) {
        hipEvent_t e = nullptr;
        HIPX(ctx, hipEventCreate(&e));
        ctx->ev_batch.push_back(e);
    }
    // the stepping kernel re-initialises its lanes itself (reset_lane in its
    // prologue): one launch per batch
    const DevResetImage R = reset_image(ctx);
    const LdsPlan plan = lds_plan(ctx);
    const int64_t kflags = (int64_t)k1_flags();
    // one event pair around the whole sequence, each batch reporting the mean:
    // timing events between the launches cost ~8 us per batch on MI355X (C2
    // 0.1765 -> 0.1688 ms per batch, scripts/gpu_ab_events.sh).  The mean includes
    // the launch gaps, so it is an upper bound of the kernel's own duration.
    // MG_BATCH_EVENTS=1 brackets every launch instead.
    const char *bev = getenv("MG_BATCH_EVENTS");
    const bool per_batch_events = bev && bev[0] == '1';
    for (uint32_t b = 0; b < n_batches; ++b) {
        if (per_batch_events || b == 0u) HIPX(ctx, hipEventRecord(ctx->ev_batch[2u * b], ctx->stream));
        int rc = launch_step(ctx, hook_mask, max_steps, max_depth, ctx->d_ctr_multi + (size_t)b * nb,
                             nullptr, 0u, &R, &plan, kflags);
        if (rc) return rc;
        if (per_batch_events || b + 1u == n_batches)
            HIPX(ctx, hipEventRecord(ctx->ev_batch[2u * b + 1u], ctx->stream));
    }
    HIPX(ctx, hipMemcpyAsync(ctx->h_ctr_pin, ctx->d_ctr_multi, slots * sizeof(DevCounters),
                             hipMemcpyDeviceToHost, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    float ms_all = 0.f;
    if (!per_batch_events) {
        HIPX(ctx, hipEventElapsedTime(&ms_all, ctx->ev_batch[0], ctx->ev_batch[2u * n_batches - 1u]));
        ms_all /= (float)n_batches;
    }
    for (uint32_t b = 0; b < n_batches; ++b) {
        DevCounters c{};
        for (uint32_t k = 0; k < nb; ++k) {
            const DevCounters &x = ctx->h_ctr_pin[(size_t)b * nb + k];
            c.lane_steps += x.lane_steps; c.running += x.running; c.halted += x.halted;
            c.hooked += x.hooked; c.escaped += x.escaped;
        }
        float ms = ms_all;
        if (per_batch_events)
            HIPX(ctx, hipEventElapsedTime(&ms, ctx->ev_batch[2u * b], ctx->ev_batch[2u * b + 1u]));
        stats[b].lane_steps = c.lane_steps;
        stats[b].running = c.running;
        stats[b].halted = c.halted;
        stats[b].hooked = c.hooked;
        stats[b].escaped = c.escaped;
        stats[b].kernel_ms = ms;
        stats[b].launches = 1;
    }
    return MG_OK;
}

extern "C" int mg_step_profile(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps, uint32_t max_depth,
                               uint64_t *op_counts, uint64_t *extra) {
    if (!ctx || !op_counts || !extra) return MG_EINVAL;
    if (!ctx->uploaded) return set_err(ctx, MG_ESTATE, "mg_step_profile before mg_lanes_upload");
    HIPX(ctx, hipSetDevice(ctx->device));
    unsigned long long *d = nullptr;
    HIPX(ctx, hipMalloc(&d, 260 * sizeof(unsigned long long)));
    hipMemsetAsync(d, 0, 260 * sizeof(unsigned long long), ctx->stream);
    int rc = launch_step(ctx, hook_mask, max_steps, max_depth, nullptr, d);
    unsigned long long h[260];
    if (!rc) {
        hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, ctx->stream);
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) rc = set_err(ctx, MG_EDEVICE, "profile step: %s", hipGetErrorString(e));
    }
    hipFree(d);
    if (rc) return rc;
    for (int i = 0; i < 256; ++i) op_counts[i] = h[i];
    for (int i = 0; i < 4; ++i) extra[i] = h[256 + i];
    return MG_OK;
}

extern "C" int mg_step_async(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps, uint32_t max_depth) {
    if (!ctx) return MG_EINVAL;
    if (!ctx->uploaded) return set_err(ctx, MG_ESTATE, "mg_step_async before mg_lanes_upload");
    return launch_step(ctx, hook_mask, max_steps, max_depth, nullptr);
}

extern "C" int mg_sync(mg_ctx *ctx) {
    if (!ctx) return MG_EINVAL;
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

extern "C" int mg_coverage(mg_ctx *ctx, uint32_t code_id, uint8_t *bytes, uint32_t n) {
    if (!ctx || code_id >= ctx->codes.size()) return set_err(ctx, MG_ENOCODE, "unknown code_id");
    const DevCode &c = ctx->codes[code_id];
    if (!bytes || n < c.n_instr) return set_err(ctx, MG_EINVAL, "coverage buffer too small");
    HIPX(ctx, hipMemcpyAsync(bytes, ctx->d_cov + c.cov_off, c.n_instr, hipMemcpyDeviceToHost, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

extern "C" int mg_coverage_clear(mg_ctx *ctx) {
    if (!ctx) return MG_EINVAL;
    if (ctx->d_cov) HIPX(ctx, hipMemsetAsync(ctx->d_cov, 0, ctx->cap_cov, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

extern "C" int mg_event_counts(mg_ctx *ctx, uint32_t *sha3_count, uint32_t *exp_count, uint32_t first, uint32_t n) {
    if (!ctx || !ctx->have_lanes || first + (uint64_t)n > ctx->L.n) return set_err(ctx, MG_EINVAL, "bad lane range");
    if (sha3_count) HIPX(ctx, hipMemcpyAsync(sha3_count, ctx->L.sha3_count + first, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (exp_count) HIPX(ctx, hipMemcpyAsync(exp_count, ctx->L.exp_count + first, (size_t)n * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPX(ctx, hipStreamSynchronize(ctx->stream));
    return MG_OK;
}

// ----------------------------------------------------------- kernel 2 C-ABI
extern "C" int mg_eval_upload(mg_ctx *ctx, const mg_dag_batch *dags, const mg_model_batch *models) {
    if (!ctx || !dags || !models) return MG_EINVAL;
    HIPX(ctx, hipSetDevice(ctx->device));
    std::string msg;
    const int rc = bv_upload(ctx->bv, dags, models, ctx->stream, msg);
    if (rc) return set_err(ctx, rc, "%s", msg.c_str());
    return MG_OK;
}

extern "C" int mg_eval_run(mg_ctx *ctx, uint32_t dag_first, uint32_t dag_count, float *kernel_ms) {
    if (!ctx) return MG_EINVAL;
    HIPX(ctx, hipSetDevice(ctx->device));
    std::string msg;
    if (kernel_ms) HIPX(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    const int rc = bv_run(ctx->bv, dag_first, dag_count, ctx->stream, msg);
    if (rc) return set_err(ctx, rc, "%s", msg.c_str());
    if (kernel_ms) {
        HIPX(ctx, hipEventRecord(ctx->ev1, ctx->stream));
        HIPX(ctx, hipEventSynchronize(ctx->ev1));
        HIPX(ctx, hipEventElapsedTime(kernel_ms, ctx->ev0, ctx->ev1));
    }
    return MG_OK;
}

extern "C" int mg_eval_download(mg_ctx *ctx, uint32_t *first_sat, uint32_t *sat_count, uint32_t dag_first,
                                uint32_t dag_count) {
    if (!ctx) return MG_EINVAL;
    std::string msg;
    const int rc = bv_download(ctx->bv, first_sat, sat_count, dag_first, dag_count, ctx->stream, msg);
    if (rc) return set_err(ctx, rc, "%s", msg.c_str());
    return MG_OK;
}

extern "C" int mg_eval_bits(mg_ctx *ctx, const mg_dag_batch *dags, const mg_model_batch *models,
                            uint32_t *first_sat, uint32_t *sat_count, uint64_t *sat_bits, float *kernel_ms) {
    if (!ctx || !dags || !models || !sat_bits) return MG_EINVAL;
    int rc;
    if ((rc = mg_eval_upload(ctx, dags, models))) return rc;
    ctx->bv.want_bits = true;
    rc = mg_eval_run(ctx, 0, dags->n_dags, kernel_ms);
    if (!rc) {
        std::string msg;
        rc = bv_download(ctx->bv, first_sat, sat_count, 0, dags->n_dags, ctx->stream, msg,
                         (unsigned long long *)sat_bits);
        if (rc) set_err(ctx, rc, "%s", msg.c_str());
    }
    ctx->bv.want_bits = false;
    return rc;
}

extern "C" int mg_eval(mg_ctx *ctx, const mg_dag_batch *dags, const mg_model_batch *models, uint32_t *first_sat,
                       uint32_t *sat_count, float *kernel_ms) {
    int rc;
    if ((rc = mg_eval_upload(ctx, dags, models))) return rc;
    if ((rc = mg_eval_run(ctx, 0, dags->n_dags, kernel_ms))) return rc;
    return mg_eval_download(ctx, first_sat, sat_count, 0, dags->n_dags);
}

// ------------------------------------------------------------ conjunct compiler
// mg_cc_*: kernel 2's program compiler on the host, over a growing native node
// table (csrc/cc.h; the passes of mythril_amd/smt/flatten.py).
struct mg_cc {
    mgcc::Compiler c;
    std::vector<uint32_t> buf;
};

extern "C" int mg_cc_open(mg_cc **out) {
    if (!out) return MG_EINVAL;
    *out = new (std::nothrow) mg_cc();
    return *out ? MG_OK : MG_ENOMEM;
}

extern "C" void mg_cc_close(mg_cc *cc) { delete cc; }

extern "C" const char *mg_cc_error(mg_cc *cc) { return cc ? cc->c.err.c_str() : "null compiler"; }

extern "C" int mg_cc_add(mg_cc *cc, const uint32_t *rows, uint32_t n, const uint32_t *args, uint32_t n_args,
                         uint32_t *ids) {
    if (!cc || (n && (!rows || !ids))) return MG_EINVAL;
    return cc->c.add(rows, n, args, n_args, ids) ? MG_EINVAL : MG_OK;
}

extern "C" int mg_cc_compile(mg_cc *cc, uint32_t root, uint32_t *insns, uint32_t cap, uint32_t *n_insns,
                             uint32_t *max_slots) {
    if (!cc || !n_insns || !max_slots) return MG_EINVAL;
    uint32_t ms = *max_slots;
    const int n = cc->c.compile(root, cc->buf, ms);
    if (n < 0) return MG_EUNSUPPORTED;
    *n_insns = (uint32_t)n;
    if ((uint32_t)n > cap || !insns) { cc->c.err = "instruction buffer too small"; return MG_EINVAL; }
    std::memcpy(insns, cc->buf.data(), (size_t)n * 4 * sizeof(uint32_t));
    *max_slots = ms;
    return MG_OK;
}
