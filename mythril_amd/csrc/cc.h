// Native conjunct compiler: kernel 2's register programs from lowered
// expression DAGs (host code, part of libmythgpu.so; C-ABI mg_cc_* in
// include/mythgpu.h).
//
// The host registers the nodes of lowered constraint DAGs once each (ids only
// grow: a DAG shared by many conjuncts -- a calldata word, a store chain -- is
// sent once), then asks for the program of one conjunct at a time.  The passes
// are mythril_amd/smt/flatten.py's, run over the native node table:
//   fold   ite(cmp(x, y), x, y) -> min/max; ite(x == y, x, y) -> y (interned)
//   emit   post-order, larger operand subtrees first, the conjunction of the
//          root folded conjunct by conjunct into one running result
//   slots  a result stays in the accumulator when its only reader is the next
//          instruction at an operand the accumulator may take (operand A, or B
//          of a commutative / swappable op), else a slot (linear scan, <= 16)
//   encode 4 x u32 per instruction (bv_eval.cuh)
// Ties between equal-size subtrees go to the lower node id (the Python pass
// breaks them by set order); every program computes the same truth value.
#pragma once

#include <algorithm>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace mgcc {

// device opcodes (mythril_amd/smt/program.py OPS) the passes name
enum : uint32_t {
    O_COPY = 0, O_ADD = 1, O_SUB = 2, O_MUL = 3, O_AND_BV = 9, O_OR_BV = 10, O_XOR_BV = 11,
    O_EQ = 17, O_ULT = 18, O_ULE = 19, O_UGT = 20, O_UGE = 21, O_SLT = 22, O_SLE = 23, O_SGT = 24, O_SGE = 25,
    O_AND = 26, O_OR = 27, O_XOR = 28, O_NOT = 29, O_IMPLIES = 30, O_ITE = 31, O_EXTRACT = 32, O_CONCAT = 33,
    O_ZEXT = 34, O_SEXT = 35, O_ADD_NOOVFL = 36, O_MUL_NOOVFL = 37, O_SUB_NOUDFL = 38, O_DISTINCT = 39,
    O_TAB = 40, O_UMIN = 41, O_UMAX = 42, O_SMIN = 43, O_SMAX = 44, O_RSUB = 45, O_RCONCAT = 46,
    N_DEVICE_OPS = 47,
    O_VAR = 0x1000, O_CONST = 0x1001,
};
constexpr uint32_t MAX_SLOTS = 16, TILE_INSNS = 2048, WMAX = 256;
constexpr uint32_t REF_ACC = 0, REF_SLOT = 1, REF_VAR = 2, REF_CONST = 3;
constexpr uint32_t NONE = 0xffffffffu;

inline bool is_cmp(uint32_t op) {
    return op == O_EQ || op == O_DISTINCT || (op >= O_ULT && op <= O_SGE) || op == O_ADD_NOOVFL ||
           op == O_MUL_NOOVFL || op == O_SUB_NOUDFL;
}
inline bool commutative(uint32_t op) {
    switch (op) {
    case O_ADD: case O_MUL: case O_AND_BV: case O_OR_BV: case O_XOR_BV: case O_EQ: case O_DISTINCT:
    case O_AND: case O_OR: case O_XOR: case O_ADD_NOOVFL: case O_MUL_NOOVFL:
    case O_UMIN: case O_UMAX: case O_SMIN: case O_SMAX:
        return true;
    default:
        return false;
    }
}
// operand-swapped form (NONE: none)
inline uint32_t swapped(uint32_t op) {
    switch (op) {
    case O_ULT: return O_UGT; case O_UGT: return O_ULT; case O_ULE: return O_UGE; case O_UGE: return O_ULE;
    case O_SLT: return O_SGT; case O_SGT: return O_SLT; case O_SLE: return O_SGE; case O_SGE: return O_SLE;
    case O_SUB: return O_RSUB; case O_RSUB: return O_SUB; case O_CONCAT: return O_RCONCAT;
    case O_RCONCAT: return O_CONCAT;
    default: return NONE;
    }
}
inline bool acc_ok(uint32_t op, uint32_t k) { return k == 0 || (k == 1 && (commutative(op) || swapped(op) != NONE)); }

struct Node {
    uint32_t op, width, a0, n, imm;     // args: Compiler::args[a0 .. a0 + n)
};

struct Key {
    uint32_t op, width, imm;
    std::vector<uint32_t> args;
    bool operator==(const Key &o) const { return op == o.op && width == o.width && imm == o.imm && args == o.args; }
};
struct KeyHash {
    size_t operator()(const Key &k) const {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](uint64_t x) { h ^= x; h *= 1099511628211ull; };
        mix(k.op); mix(k.width); mix(k.imm);
        for (uint32_t a : k.args) mix(a);
        return (size_t)h;
    }
};

struct Virt {
    uint32_t op, width, imm;
    uint32_t nargs;
    // an operand: a leaf node id (is_virt = false) or an earlier instruction
    uint32_t arg[3];
    bool is_virt[3];
};

struct Compiler {
    std::vector<Node> nodes;
    std::vector<uint32_t> args;
    std::unordered_map<Key, uint32_t, KeyHash> intern;
    std::vector<uint32_t> fold_of;      // node -> folded node (NONE: not yet)
    std::vector<uint64_t> size_of;      // node -> operand-tree size + 1 (0: not yet)
    std::string err;

    uint32_t arg(uint32_t id, uint32_t k) const { return args[nodes[id].a0 + k]; }
    bool leaf(uint32_t id) const { return nodes[id].op == O_VAR || nodes[id].op == O_CONST; }

    uint32_t make(uint32_t op, uint32_t width, uint32_t imm, const std::vector<uint32_t> &a) {
        Key k{op, width, imm, a};
        auto it = intern.find(k);
        if (it != intern.end()) return it->second;
        const uint32_t id = (uint32_t)nodes.size();
        nodes.push_back(Node{op, width, (uint32_t)args.size(), (uint32_t)a.size(), imm});
        args.insert(args.end(), a.begin(), a.end());
        intern.emplace(std::move(k), id);
        fold_of.push_back(NONE);
        size_of.push_back(0);
        return id;
    }

    // rows: {op, width, first_arg, nargs, imm} x n; an argument is a node id, or
    // 0x80000000 | k for the k-th row of this same call.  ids[i] receives row i's
    // node id (an existing id when an equal node exists already: folding can
    // create a node the host registers later)
    int add(const uint32_t *rows, uint32_t n, const uint32_t *a, uint32_t na, uint32_t *ids) {
        std::vector<uint32_t> av;
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t *r = rows + 5 * i;
            if (r[2] + (uint64_t)r[3] > na) { err = "argument range out of bounds"; return -1; }
            av.assign(a + r[2], a + r[2] + r[3]);
            for (uint32_t &x : av) {
                if (x & 0x80000000u) {
                    const uint32_t k = x & 0x7fffffffu;
                    if (k >= i) { err = "argument refers to a later row"; return -1; }
                    x = ids[k];
                } else if (x >= nodes.size()) {
                    err = "argument refers to an unregistered node";
                    return -1;
                }
            }
            ids[i] = make(r[0], r[1], r[4], av);
        }
        return 0;
    }

    // flatten._fold_select
    uint32_t fold(uint32_t root) {
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            auto [x, ready] = st.back();
            st.pop_back();
            if (fold_of[x] != NONE) continue;
            const Node nd = nodes[x];
            if (nd.n == 0) { fold_of[x] = x; continue; }
            if (!ready) {
                st.push_back({x, true});
                for (uint32_t k = 0; k < nd.n; ++k)
                    if (fold_of[arg(x, k)] == NONE) st.push_back({arg(x, k), false});
                continue;
            }
            std::vector<uint32_t> a(nd.n);
            bool same = true;
            for (uint32_t k = 0; k < nd.n; ++k) { a[k] = fold_of[arg(x, k)]; same &= a[k] == arg(x, k); }
            uint32_t out = same ? x : make(nd.op, nd.width, nd.imm, a);
            if (nd.op == O_ITE && nd.width > 1) {
                const uint32_t c = a[0], p = a[1], q = a[2];
                const uint32_t cop = nodes[c].op;
                const bool minmax = cop >= O_ULT && cop <= O_SGE;
                if ((minmax || cop == O_EQ) && nodes[c].n == 2) {
                    const uint32_t cx = arg(c, 0), cy = arg(c, 1);
                    const bool fwd = cx == p && cy == q, rev = cy == p && cx == q;
                    if (fwd || rev) {
                        if (cop == O_EQ) {
                            out = q;
                        } else {
                            // (lo, hi) op per compare: ult/ule -> (umin, umax), ugt/uge ->
                            // (umax, umin), slt/sle -> (smin, smax), sgt/sge -> (smax, smin)
                            uint32_t lo, hi;
                            switch (cop) {
                            case O_ULT: case O_ULE: lo = O_UMIN; hi = O_UMAX; break;
                            case O_UGT: case O_UGE: lo = O_UMAX; hi = O_UMIN; break;
                            case O_SLT: case O_SLE: lo = O_SMIN; hi = O_SMAX; break;
                            default: lo = O_SMAX; hi = O_SMIN; break;
                            }
                            out = make(fwd ? lo : hi, nd.width, 0, {cx, cy});
                        }
                    }
                }
            }
            fold_of[x] = out;
            if (fold_of[out] == NONE) fold_of[out] = out;     // a folded node folds to itself
        }
        return fold_of[root];
    }

    uint64_t size(uint32_t root) {
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            auto [x, ready] = st.back();
            st.pop_back();
            if (size_of[x] || leaf(x)) continue;
            if (!ready) {
                st.push_back({x, true});
                for (uint32_t k = 0; k < nodes[x].n; ++k) st.push_back({arg(x, k), false});
                continue;
            }
            uint64_t s = 1;                     // tree size (shared operands counted per use)
            for (uint32_t k = 0; k < nodes[x].n; ++k) {
                const uint32_t c = arg(x, k);
                const uint64_t sc = leaf(c) ? 0 : size_of[c] - 1;
                s = s + sc < s ? ~0ull - 1 : s + sc;    // saturating
            }
            size_of[x] = s + 1;                 // stored + 1 (0 = not yet)
        }
        return leaf(root) ? 0 : size_of[root] - 1;
    }
    uint64_t sz(uint32_t id) { return leaf(id) ? 0 : size(id); }

    // flatten.Compiler._lower for one node; returns false (err set) when unsupported
    bool lower_virt(uint32_t x, std::vector<Virt> &vs, std::unordered_map<uint32_t, uint32_t> &vid) {
        const Node nd = nodes[x];
        auto opnd = [&](Virt &v, uint32_t k, uint32_t c) {
            auto it = vid.find(c);
            if (it != vid.end()) { v.arg[k] = it->second; v.is_virt[k] = true; }
            else { v.arg[k] = c; v.is_virt[k] = false; }
        };
        if ((nd.op == O_AND || nd.op == O_OR) && nd.n > 2) {
            Virt v{nd.op, 1, 0, 2, {0, 0, 0}, {false, false, false}};
            opnd(v, 0, arg(x, 0));
            for (uint32_t k = 1; k < nd.n; ++k) {
                opnd(v, 1, arg(x, k));
                vs.push_back(v);
                v.arg[0] = (uint32_t)vs.size() - 1;
                v.is_virt[0] = true;
            }
            vid[x] = (uint32_t)vs.size() - 1;
            return true;
        }
        Virt v{nd.op, nd.width, 0, nd.n, {0, 0, 0}, {false, false, false}};
        if (nd.n > 3) { err = "operation with more than three operands"; return false; }
        if ((nd.op == O_AND || nd.op == O_OR) && nd.n == 1) {
            v.op = O_COPY;
            v.width = 1;
        } else if (nd.op == O_ZEXT && vid.count(arg(x, 0))) {
            vid[x] = vid[arg(x, 0)];            // values are kept masked: the same instruction
            return true;
        } else if (nd.op == O_EXTRACT) {
            v.imm = nd.imm;                      // low bit
        } else if (nd.op == O_SEXT) {
            v.imm = nodes[arg(x, 0)].width;
        } else if (nd.op == O_CONCAT) {
            v.imm = nodes[arg(x, 1)].width;
        } else if (is_cmp(nd.op)) {
            v.width = 1;
            v.imm = nodes[arg(x, 0)].width;
        } else if (nd.op == O_TAB) {
            v.imm = nd.imm;
        } else if (nd.op >= N_DEVICE_OPS) {
            err = "operation not evaluated on the device";
            return false;
        }
        for (uint32_t k = 0; k < nd.n; ++k) opnd(v, k, arg(x, k));
        vs.push_back(v);
        vid[x] = (uint32_t)vs.size() - 1;
        return true;
    }

    bool emit(uint32_t n, std::vector<Virt> &vs, std::unordered_map<uint32_t, uint32_t> &vid) {
        std::vector<std::pair<uint32_t, bool>> st{{n, false}};
        std::vector<uint32_t> kids;
        while (!st.empty()) {
            auto [x, ready] = st.back();
            st.pop_back();
            if (vid.count(x) || leaf(x)) continue;
            const Node nd = nodes[x];
            bool wide = nd.width > WMAX;
            for (uint32_t k = 0; k < nd.n; ++k) wide |= nodes[arg(x, k)].width > WMAX;
            if (wide) { err = "bit-vector wider than 256 bits"; return false; }
            if (!ready) {
                st.push_back({x, true});
                kids.clear();
                for (uint32_t k = 0; k < nd.n; ++k) {
                    const uint32_t c = arg(x, k);
                    if (!vid.count(c) && !leaf(c) && std::find(kids.begin(), kids.end(), c) == kids.end())
                        kids.push_back(c);
                }
                // ascending size (ties: lower id first), pushed smallest-first => computed largest-first
                std::sort(kids.begin(), kids.end(), [&](uint32_t a, uint32_t b) {
                    const uint64_t sa = sz(a), sb = sz(b);
                    return sa != sb ? sa < sb : a < b;
                });
                for (uint32_t c : kids) st.push_back({c, false});
                continue;
            }
            if (!lower_virt(x, vs, vid)) return false;
        }
        return true;
    }

    // returns the number of instructions, or -1 (unsupported, err set)
    int compile(uint32_t root0, std::vector<uint32_t> &out, uint32_t &max_slot) {
        if (root0 >= nodes.size()) { err = "unknown root"; return -1; }
        const uint32_t root = fold(root0);
        std::vector<Virt> vs;
        std::unordered_map<uint32_t, uint32_t> vid;
        std::vector<uint32_t> conj;
        if (nodes[root].op == O_AND) for (uint32_t k = 0; k < nodes[root].n; ++k) conj.push_back(arg(root, k));
        else conj.push_back(root);
        bool have = false;
        uint32_t run = 0;
        bool run_virt = false;
        for (uint32_t c : conj) {
            if (!emit(c, vs, vid)) return -1;
            uint32_t cur;
            bool cur_virt;
            auto it = vid.find(c);
            if (it != vid.end()) { cur = it->second; cur_virt = true; }
            else { cur = c; cur_virt = false; }
            if (!have) {
                if (!cur_virt) {
                    Virt v{O_COPY, nodes[c].width, 0, 1, {c, 0, 0}, {false, false, false}};
                    vs.push_back(v);
                    cur = (uint32_t)vs.size() - 1;
                    cur_virt = true;
                }
                run = cur; run_virt = cur_virt; have = true;
            } else {
                Virt v{O_AND, 1, 0, 2, {run, cur, 0}, {run_virt, cur_virt, false}};
                vs.push_back(v);
                run = (uint32_t)vs.size() - 1;
                run_virt = true;
            }
        }
        const uint32_t n = (uint32_t)vs.size();
        if (n > TILE_INSNS) { err = "program longer than one LDS tile"; return -1; }
        // uses of each instruction's result
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> uses(n);
        for (uint32_t i = 0; i < n; ++i)
            for (uint32_t k = 0; k < vs[i].nargs; ++k)
                if (vs[i].is_virt[k]) uses[vs[i].arg[k]].push_back({i, k});
        std::vector<uint32_t> slot_of(n, NONE), last_use(n, 0);
        std::vector<bool> needs(n, false);
        for (uint32_t j = 0; j < n; ++j) {
            if (uses[j].empty()) continue;
            bool need = uses[j].size() > 1;
            for (auto [i, k] : uses[j]) {
                need |= i != j + 1 || !acc_ok(vs[i].op, k);
                last_use[j] = std::max(last_use[j], i);
            }
            needs[j] = need;
        }
        std::vector<uint32_t> free_slots;
        for (int s = (int)MAX_SLOTS - 1; s >= 0; --s) free_slots.push_back((uint32_t)s);
        std::vector<std::vector<uint32_t>> expiring(n + 2);
        for (uint32_t i = 0; i < n; ++i) {
            for (uint32_t s : expiring[i]) free_slots.push_back(s);
            expiring[i].clear();
            if (!needs[i]) continue;
            if (free_slots.empty()) { err = "constraint set needs more than 16 live values"; return -1; }
            const uint32_t s = free_slots.back();
            free_slots.pop_back();
            slot_of[i] = s;
            max_slot = std::max(max_slot, s + 1);
            expiring[last_use[i] + 1].push_back(s);
        }
        out.assign((size_t)n * 4, 0u);
        for (uint32_t i = 0; i < n; ++i) {
            const Virt &v = vs[i];
            uint32_t refs[3] = {0, 0, 0};
            bool is_acc[3] = {false, false, false};
            for (uint32_t k = 0; k < v.nargs; ++k) {
                if (v.is_virt[k]) {
                    const uint32_t j = v.arg[k];
                    const bool acc = j + 1 == i && (k == 0 || slot_of[j] == NONE);
                    refs[k] = acc ? (REF_ACC << 30) : ((REF_SLOT << 30) | slot_of[j]);
                    is_acc[k] = acc;
                } else {
                    const Node &lf = nodes[v.arg[k]];
                    refs[k] = ((lf.op == O_CONST ? REF_CONST : REF_VAR) << 30) | lf.imm;
                }
            }
            uint32_t op = v.op;
            if (v.nargs > 1 && is_acc[1]) {
                std::swap(refs[0], refs[1]);
                std::swap(is_acc[0], is_acc[1]);
                if (!commutative(op)) op = swapped(op);
            }
            for (uint32_t k = 1; k < v.nargs; ++k)
                if (is_acc[k]) { err = "accumulator past operand A"; return -1; }
            uint32_t w0 = op | (v.width << 8);
            if (slot_of[i] != NONE) w0 |= (1u << 17) | (slot_of[i] << 18);
            uint32_t *w = &out[(size_t)i * 4];
            w[0] = w0;
            for (uint32_t k = 0; k < v.nargs; ++k) w[1 + k] = refs[k];
            if (v.op == O_EXTRACT || v.op == O_SEXT) w[2] = v.imm;
            else if (v.op == O_CONCAT || v.op == O_RCONCAT || is_cmp(v.op) || v.op == O_TAB) w[3] = v.imm;
        }
        return (int)n;
    }
};

}  // namespace mgcc
