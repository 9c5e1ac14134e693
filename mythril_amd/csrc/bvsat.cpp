// bvsat.cpp — the exact decision procedure behind kernel 2 (include/mythsmt.h).
//
// Kernel 2 answers a path-constraint query with a model when one of its
// candidates satisfies it; the SAT-only search tries more candidates; neither
// can say "unsat".  The reference answers those queries with z3
// (support/model.py:37-82: Optimize().check() -> sat / unsat / timeout, and
// is_possible maps unsat and timeout to "prune", state/constraints.py:33-43).
// This file decides them: the query DAG is bit-blasted into CNF (Tseitin over
// structurally hashed AND/XOR/MUX gates with constant folding), arrays are
// expanded along their store chains with Ackermann constraints between the
// reads of each base array, uninterpreted functions (keccak256_N, its inverse
// keccak256_N-1, Power) get Ackermann congruence between their applications,
// and a CDCL solver (two watched literals, 1-UIP learning with clause
// minimisation, VSIDS, phase saving, Luby restarts, activity-based clause
// deletion, assumptions) decides the CNF within a conflict / wall-clock budget.
// z3's `minimize` objectives (analysis/solver.py:219-259) are met
// lexicographically, bit by bit from the most significant, under assumptions.
//
// Bit-vector semantics are SMT-LIB's: division by zero
// gives all-ones (udiv), the dividend (urem, srem, smod), 1 or -1 (sdiv);
// shifts by >= width give 0 or the sign fill.  Host code only: no GPU here.
#include "../../include/mythsmt.h"

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

typedef int Lit;                       // 2 * var + negated
inline Lit mk(int v, bool n = false) { return 2 * v + (n ? 1 : 0); }
inline Lit neg(Lit l) { return l ^ 1; }
inline int var(Lit l) { return l >> 1; }
inline bool sgn(Lit l) { return l & 1; }
const int8_t LF = 0, LT = 1, LU = 2;
const uint32_t CR_NONE = 0xffffffffu;

// ---------------------------------------------------------------- CDCL core
struct Watcher {
    uint32_t cref;
    Lit blocker;
};

class Sat {
public:
    std::vector<uint32_t> arena;       // clause: [size | learnt << 31][activity bits][lits...]
    std::vector<uint32_t> learnts;
    std::vector<std::vector<Watcher>> watches;
    std::vector<int8_t> assigns;
    std::vector<int8_t> phase;
    std::vector<int> level;
    std::vector<uint32_t> reason;
    std::vector<double> activity;
    std::vector<char> seen;
    std::vector<Lit> trail;
    std::vector<int> trail_lim;
    std::vector<int> heap, heap_pos;   // VSIDS max-heap over variables
    size_t qhead = 0;
    double var_inc = 1.0, cla_inc = 1.0;
    bool ok = true;
    uint64_t conflicts = 0, decisions = 0, propagations = 0, n_clauses = 0;
    std::vector<int8_t> model;

    int new_var() {
        int v = (int)assigns.size();
        assigns.push_back(LU);
        phase.push_back(1);             // first guess: false (sign set)
        level.push_back(0);
        reason.push_back(CR_NONE);
        activity.push_back(0.0);
        seen.push_back(0);
        watches.emplace_back();
        watches.emplace_back();
        heap_pos.push_back(-1);
        heap_insert(v);
        return v;
    }
    int n_vars() const { return (int)assigns.size(); }
    int8_t value(Lit l) const {
        int8_t a = assigns[var(l)];
        return a == LU ? LU : (int8_t)(a ^ (int8_t)sgn(l));
    }
    int decision_level() const { return (int)trail_lim.size(); }

    // -- heap
    bool heap_lt(int a, int b) const { return activity[a] > activity[b]; }
    void heap_up(int i) {
        int v = heap[i];
        while (i > 0) {
            int p = (i - 1) >> 1;
            if (!heap_lt(v, heap[p])) break;
            heap[i] = heap[p];
            heap_pos[heap[i]] = i;
            i = p;
        }
        heap[i] = v;
        heap_pos[v] = i;
    }
    void heap_down(int i) {
        int v = heap[i], n = (int)heap.size();
        for (;;) {
            int c = 2 * i + 1;
            if (c >= n) break;
            if (c + 1 < n && heap_lt(heap[c + 1], heap[c])) ++c;
            if (!heap_lt(heap[c], v)) break;
            heap[i] = heap[c];
            heap_pos[heap[i]] = i;
            i = c;
        }
        heap[i] = v;
        heap_pos[v] = i;
    }
    void heap_insert(int v) {
        if (heap_pos[v] >= 0) return;
        heap.push_back(v);
        heap_pos[v] = (int)heap.size() - 1;
        heap_up((int)heap.size() - 1);
    }
    int heap_pop() {
        int v = heap[0];
        heap[0] = heap.back();
        heap_pos[heap[0]] = 0;
        heap.pop_back();
        heap_pos[v] = -1;
        if (!heap.empty()) heap_down(0);
        return v;
    }
    void bump_var(int v) {
        if ((activity[v] += var_inc) > 1e100) {
            for (double &a : activity) a *= 1e-100;
            var_inc *= 1e-100;
        }
        if (heap_pos[v] >= 0) heap_up(heap_pos[v]);
    }

    // -- clauses
    uint32_t csize(uint32_t c) const { return arena[c] & 0x3fffffffu; }
    bool clearnt(uint32_t c) const { return (arena[c] >> 31) != 0; }
    bool cdeleted(uint32_t c) const { return ((arena[c] >> 30) & 1u) != 0; }
    float &cact(uint32_t c) { return *reinterpret_cast<float *>(&arena[c + 1]); }
    Lit *clits(uint32_t c) { return reinterpret_cast<Lit *>(&arena[c + 2]); }
    uint32_t alloc(const std::vector<Lit> &ls, bool learnt) {
        uint32_t c = (uint32_t)arena.size();
        arena.push_back((uint32_t)ls.size() | (learnt ? 0x80000000u : 0u));
        float a = 0.f;
        uint32_t ab;
        std::memcpy(&ab, &a, 4);
        arena.push_back(ab);
        for (Lit l : ls) arena.push_back((uint32_t)l);
        return c;
    }
    void attach(uint32_t c) {
        Lit *ls = clits(c);
        watches[neg(ls[0])].push_back({c, ls[1]});
        watches[neg(ls[1])].push_back({c, ls[0]});
    }
    void enqueue(Lit p, uint32_t from) {
        assigns[var(p)] = (int8_t)!sgn(p);
        level[var(p)] = decision_level();
        reason[var(p)] = from;
        trail.push_back(p);
    }

    // Level-0 clause: simplified against the current level-0 assignment (scratch
    // buffers: clause construction allocates nothing once they have grown).
    std::vector<Lit> cl_in, cl_out;
    bool add_clause(std::initializer_list<Lit> ls) { return add_clause(ls.begin(), ls.size()); }
    bool add_clause(const std::vector<Lit> &ls) { return add_clause(ls.data(), ls.size()); }
    bool add_clause(const Lit *ls, size_t n) {
        if (!ok) return false;
        cl_in.assign(ls, ls + n);
        std::sort(cl_in.begin(), cl_in.end());
        cl_out.clear();
        Lit prev = -1;
        for (Lit l : cl_in) {
            if (value(l) == LT || l == neg(prev)) return true;
            if (value(l) != LF && l != prev) cl_out.push_back(l);
            prev = l;
        }
        ++n_clauses;
        if (cl_out.empty()) return ok = false;
        if (cl_out.size() == 1) {
            enqueue(cl_out[0], CR_NONE);
            return ok = (propagate() == CR_NONE);
        }
        attach(alloc(cl_out, false));
        return true;
    }

    uint32_t propagate() {
        uint32_t confl = CR_NONE;
        while (qhead < trail.size()) {
            Lit p = trail[qhead++];
            std::vector<Watcher> &ws = watches[p];
            Lit false_lit = neg(p);
            size_t i = 0, j = 0, n = ws.size();
            ++propagations;
            while (i < n) {
                Watcher w = ws[i];
                if (value(w.blocker) == LT) { ws[j++] = ws[i++]; continue; }
                uint32_t c = w.cref;
                Lit *ls = clits(c);
                if (ls[0] == false_lit) { ls[0] = ls[1]; ls[1] = false_lit; }
                ++i;
                Lit first = ls[0];
                if (first != w.blocker && value(first) == LT) { ws[j++] = {c, first}; continue; }
                uint32_t sz = csize(c);
                bool found = false;
                for (uint32_t k = 2; k < sz; ++k) {
                    if (value(ls[k]) != LF) {
                        ls[1] = ls[k];
                        ls[k] = false_lit;
                        watches[neg(ls[1])].push_back({c, first});
                        found = true;
                        break;
                    }
                }
                if (found) continue;
                ws[j++] = {c, first};
                if (value(first) == LF) {
                    confl = c;
                    qhead = trail.size();
                    while (i < n) ws[j++] = ws[i++];
                } else {
                    enqueue(first, c);
                }
            }
            ws.resize(j);
        }
        return confl;
    }

    void cancel_until(int lvl) {
        if (decision_level() <= lvl) return;
        for (int c = (int)trail.size() - 1; c >= trail_lim[lvl]; --c) {
            int v = var(trail[c]);
            phase[v] = (int8_t)sgn(trail[c]);
            assigns[v] = LU;
            reason[v] = CR_NONE;
            if (rel.empty() || (v < (int)rel.size() && rel[v])) heap_insert(v);
        }
        trail.resize(trail_lim[lvl]);
        trail_lim.resize(lvl);
        qhead = trail.size();
    }

    void analyze(uint32_t confl, std::vector<Lit> &out, int &bt) {
        out.clear();
        out.push_back(-1);
        int path = 0;
        Lit p = -1;
        int index = (int)trail.size() - 1;
        std::vector<int> touched;
        do {
            if (clearnt(confl)) {
                float &a = cact(confl);
                if ((a += (float)cla_inc) > 1e20f) {
                    for (uint32_t l : learnts) cact(l) *= 1e-20f;
                    cla_inc *= 1e-20;
                }
            }
            Lit *ls = clits(confl);
            uint32_t sz = csize(confl);
            for (uint32_t j = (p == -1) ? 0 : 1; j < sz; ++j) {
                Lit q = ls[j];
                int v = var(q);
                if (!seen[v] && level[v] > 0) {
                    bump_var(v);
                    seen[v] = 1;
                    touched.push_back(v);
                    if (level[v] >= decision_level()) ++path;
                    else out.push_back(q);
                }
            }
            while (!seen[var(trail[index--])]) {}
            p = trail[index + 1];
            confl = reason[var(p)];
            seen[var(p)] = 0;
            --path;
        } while (path > 0);
        out[0] = neg(p);
        // local minimisation: drop a literal implied by others of the clause
        size_t k = 1;
        for (size_t i = 1; i < out.size(); ++i) {
            uint32_t r = reason[var(out[i])];
            bool keep = true;
            if (r != CR_NONE) {
                keep = false;
                Lit *ls = clits(r);
                for (uint32_t j = 1; j < csize(r); ++j) {
                    int v = var(ls[j]);
                    if (!seen[v] && level[v] > 0) { keep = true; break; }
                }
            }
            if (keep) out[k++] = out[i];
        }
        out.resize(k);
        for (int v : touched) seen[v] = 0;
        bt = 0;
        if (out.size() > 1) {
            size_t mi = 1;
            for (size_t i = 2; i < out.size(); ++i)
                if (level[var(out[i])] > level[var(out[mi])]) mi = i;
            std::swap(out[1], out[mi]);
            bt = level[var(out[1])];
        }
    }

    bool locked(uint32_t c) {
        Lit l0 = clits(c)[0];
        return reason[var(l0)] == c && value(l0) == LT;
    }

    void reduce_db() {
        std::sort(learnts.begin(), learnts.end(), [&](uint32_t a, uint32_t b) {
            uint32_t sa = csize(a), sb = csize(b);
            if ((sa > 2) != (sb > 2)) return sb <= 2;
            return cact(a) < cact(b);
        });
        size_t half = learnts.size() / 2, k = 0;
        for (size_t i = 0; i < learnts.size(); ++i) {
            uint32_t c = learnts[i];
            if (i < half && csize(c) > 2 && !locked(c)) arena[c] |= 0x40000000u;
            else learnts[k++] = c;
        }
        learnts.resize(k);
        for (auto &ws : watches) {
            size_t j = 0;
            for (size_t i = 0; i < ws.size(); ++i)
                if (!cdeleted(ws[i].cref)) ws[j++] = ws[i];
            ws.resize(j);
        }
    }

    static double luby(double y, int x) {
        int size = 1, seq = 0;
        while (size < x + 1) { ++seq; size = 2 * size + 1; }
        while (size - 1 != x) { size = (size - 1) >> 1; --seq; x = x % size; }
        double r = 1;
        for (int i = 0; i < seq; ++i) r *= y;
        return r;
    }

    // LT sat, LF unsat (under the assumptions), LU budget exhausted
    // Decisions over `relevant` only (a session's query: the inputs of its
    // cone -- every gate it depends on follows from them by propagation); the
    // variables of other queries' terms stay unassigned, and a SAT answer is
    // the cone's.  Empty: every variable.
    std::vector<char> rel;
    void set_relevant(const std::vector<int> *relevant) {
        for (int v : heap) heap_pos[v] = -1;
        heap.clear();
        if (!relevant) {
            rel.clear();
            for (int v = 0; v < n_vars(); ++v)
                if (assigns[v] == LU) heap_insert(v);
            return;
        }
        rel.assign(n_vars(), 0);
        for (int v : *relevant) rel[v] = 1;
        for (int v : *relevant)
            if (assigns[v] == LU) heap_insert(v);
    }

    int8_t solve(const std::vector<Lit> &assumptions, uint64_t max_conflicts,
                 std::chrono::steady_clock::time_point deadline, bool timed) {
        model.clear();
        if (!ok) return LF;
        uint64_t start = conflicts;
        double max_learnts = std::max(2000.0, n_clauses / 3.0);
        int restarts = 0;
        std::vector<Lit> learnt;
        for (;;) {
            uint64_t budget = (uint64_t)(luby(2.0, restarts++) * 100);
            uint64_t here = 0;
            for (;;) {
                uint32_t confl = propagate();
                if (confl != CR_NONE) {
                    ++conflicts;
                    ++here;
                    if (decision_level() == 0) { ok = false; return LF; }
                    int bt;
                    analyze(confl, learnt, bt);
                    cancel_until(bt);
                    if (learnt.size() == 1) {
                        enqueue(learnt[0], CR_NONE);
                    } else {
                        uint32_t c = alloc(learnt, true);
                        learnts.push_back(c);
                        attach(c);
                        cact(c) += (float)cla_inc;
                        enqueue(learnt[0], c);
                    }
                    var_inc *= 1.0 / 0.95;
                    cla_inc *= 1.0 / 0.999;
                    if ((conflicts & 255u) == 0 && timed && std::chrono::steady_clock::now() > deadline) {
                        cancel_until(0);
                        return LU;
                    }
                    if (max_conflicts && conflicts - start >= max_conflicts) {
                        cancel_until(0);
                        return LU;
                    }
                    continue;
                }
                if (here >= budget) { cancel_until(0); break; }       // restart
                if ((double)learnts.size() - (double)trail.size() >= max_learnts) {
                    reduce_db();
                    max_learnts *= 1.1;
                }
                Lit next = -1;
                while (decision_level() < (int)assumptions.size()) {
                    Lit a = assumptions[decision_level()];
                    if (value(a) == LT) {
                        trail_lim.push_back((int)trail.size());
                    } else if (value(a) == LF) {
                        cancel_until(0);
                        return LF;
                    } else {
                        next = a;
                        break;
                    }
                }
                if (next == -1) {
                    int v = -1;
                    while (!heap.empty()) {
                        int c = heap_pop();
                        if (assigns[c] == LU) { v = c; break; }
                    }
                    if (v < 0) {
                        model.assign(assigns.begin(), assigns.end());
                        cancel_until(0);
                        return LT;
                    }
                    ++decisions;
                    next = mk(v, phase[v] != 0);
                }
                trail_lim.push_back((int)trail.size());
                enqueue(next, CR_NONE);
            }
        }
    }
};

// ---------------------------------------------------------------- gates
typedef std::vector<Lit> Bits;     // little-endian: bit 0 first

struct Key3 {
    int a, b, c, k;
    bool operator==(const Key3 &o) const { return a == o.a && b == o.b && c == o.c && k == o.k; }
};
struct Key3H {
    size_t operator()(const Key3 &x) const {
        uint64_t h = (uint64_t)(uint32_t)x.a * 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)x.b * 0xC2B2AE3D27D4EB4Full ^
                     (uint64_t)(uint32_t)x.c * 0x165667B19E3779F9ull ^ (uint64_t)x.k;
        return (size_t)(h ^ (h >> 29));
    }
};

class Gates {
public:
    Sat &S;
    Lit T, F;
    std::unordered_map<Key3, Lit, Key3H> cache;
    explicit Gates(Sat &s) : S(s) {
        T = mk(S.new_var());
        F = neg(T);
        S.add_clause({T});
    }
    Lit fresh() { return mk(S.new_var()); }
    bool is_const(Lit l) const { return l == T || l == F; }
    // a literal the level-0 assignment already decides is that constant: every
    // gate is built at level 0 (no search runs while blasting), so the facts the
    // asserted conjuncts propagate fold the gates built after them
    Lit nrm(Lit l) const {
        int8_t v = S.value(l);
        return v == LT ? T : v == LF ? F : l;
    }
    Lit and2(Lit a, Lit b) {
        a = nrm(a);
        b = nrm(b);
        if (a == F || b == F || a == neg(b)) return F;
        if (a == T) return b;
        if (b == T || a == b) return a;
        if (a > b) std::swap(a, b);
        Key3 k{a, b, 0, 1};
        auto it = cache.find(k);
        if (it != cache.end()) return it->second;
        Lit o = fresh();
        S.add_clause({neg(o), a});
        S.add_clause({neg(o), b});
        S.add_clause({o, neg(a), neg(b)});
        cache.emplace(k, o);
        return o;
    }
    Lit or2(Lit a, Lit b) { return neg(and2(neg(a), neg(b))); }
    Lit xor2(Lit a, Lit b) {
        a = nrm(a);
        b = nrm(b);
        if (a == F) return b;
        if (b == F) return a;
        if (a == T) return neg(b);
        if (b == T) return neg(a);
        if (a == b) return F;
        if (a == neg(b)) return T;
        bool flip = false;
        if (sgn(a)) { a = neg(a); flip = !flip; }
        if (sgn(b)) { b = neg(b); flip = !flip; }
        if (a > b) std::swap(a, b);
        Key3 k{a, b, 0, 2};
        auto it = cache.find(k);
        Lit o;
        if (it != cache.end()) {
            o = it->second;
        } else {
            o = fresh();
            S.add_clause({neg(o), a, b});
            S.add_clause({neg(o), neg(a), neg(b)});
            S.add_clause({o, neg(a), b});
            S.add_clause({o, a, neg(b)});
            cache.emplace(k, o);
        }
        return flip ? neg(o) : o;
    }
    Lit mux(Lit s, Lit a, Lit b) {      // s ? a : b
        s = nrm(s);
        a = nrm(a);
        b = nrm(b);
        if (s == T || a == b) return a;
        if (s == F) return b;
        if (a == T && b == F) return s;
        if (a == F && b == T) return neg(s);
        if (a == T) return or2(s, b);
        if (a == F) return and2(neg(s), b);
        if (b == T) return or2(neg(s), a);
        if (b == F) return and2(s, a);
        if (a == s) return or2(s, b);
        if (a == neg(s)) return and2(neg(s), b);
        if (b == s) return and2(s, a);
        if (b == neg(s)) return or2(neg(s), a);
        if (sgn(s)) { s = neg(s); std::swap(a, b); }
        Key3 k{s, a, b, 3};
        auto it = cache.find(k);
        if (it != cache.end()) return it->second;
        Lit o = fresh();
        S.add_clause({neg(s), neg(a), o});
        S.add_clause({neg(s), a, neg(o)});
        S.add_clause({s, neg(b), o});
        S.add_clause({s, b, neg(o)});
        S.add_clause({neg(a), neg(b), o});      // redundant: helps propagation
        S.add_clause({a, b, neg(o)});
        cache.emplace(k, o);
        return o;
    }
    Lit maj(Lit a, Lit b, Lit c) {
        a = nrm(a);
        b = nrm(b);
        c = nrm(c);
        if (is_const(a)) return a == T ? or2(b, c) : and2(b, c);
        if (is_const(b)) return b == T ? or2(a, c) : and2(a, c);
        if (is_const(c)) return c == T ? or2(a, b) : and2(a, b);
        if (a == b || a == c) return a;
        if (b == c) return b;
        if (a == neg(b)) return c;
        if (a == neg(c)) return b;
        if (b == neg(c)) return a;
        Lit x[3] = {a, b, c};
        std::sort(x, x + 3);
        Key3 k{x[0], x[1], x[2], 4};
        auto it = cache.find(k);
        if (it != cache.end()) return it->second;
        Lit o = fresh();
        S.add_clause({neg(a), neg(b), o});
        S.add_clause({neg(a), neg(c), o});
        S.add_clause({neg(b), neg(c), o});
        S.add_clause({a, b, neg(o)});
        S.add_clause({a, c, neg(o)});
        S.add_clause({b, c, neg(o)});
        cache.emplace(k, o);
        return o;
    }
    Lit and_n(const std::vector<Lit> &xs) {
        std::vector<Lit> v;
        for (Lit x : xs) {
            x = nrm(x);
            if (x == F) return F;
            if (x != T) v.push_back(x);
        }
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        for (size_t i = 1; i < v.size(); ++i)
            if (v[i] == neg(v[i - 1])) return F;
        if (v.empty()) return T;
        if (v.size() == 1) return v[0];
        if (v.size() == 2) return and2(v[0], v[1]);
        Lit o = fresh();
        std::vector<Lit> big{o};
        for (Lit x : v) {
            S.add_clause({neg(o), x});
            big.push_back(neg(x));
        }
        S.add_clause(big);
        return o;
    }
    Lit or_n(const std::vector<Lit> &xs) {
        std::vector<Lit> n;
        for (Lit x : xs) n.push_back(neg(x));
        return neg(and_n(n));
    }

    // -- words
    Bits cnst(uint32_t w, const uint32_t *limbs) {
        Bits b(w);
        for (uint32_t i = 0; i < w; ++i) b[i] = ((limbs[i >> 5] >> (i & 31)) & 1u) ? T : F;
        return b;
    }
    std::vector<int> inputs;            // variables of words (not gate outputs)
    Bits fresh_word(uint32_t w) {
        Bits b(w);
        for (auto &x : b) {
            x = fresh();
            inputs.push_back(var(x));
        }
        return b;
    }
    Bits bnot(const Bits &a) {
        Bits r(a.size());
        for (size_t i = 0; i < a.size(); ++i) r[i] = neg(a[i]);
        return r;
    }
    Bits add(const Bits &a, const Bits &b, Lit cin, Lit *cout = nullptr) {
        Bits r(a.size());
        Lit c = cin;
        for (size_t i = 0; i < a.size(); ++i) {
            r[i] = xor2(xor2(a[i], b[i]), c);
            c = maj(a[i], b[i], c);
        }
        if (cout) *cout = c;
        return r;
    }
    Bits sub(const Bits &a, const Bits &b) { return add(a, bnot(b), T); }
    Bits bneg(const Bits &a) { return add(Bits(a.size(), F), bnot(a), T); }
    Lit eq(const Bits &a, const Bits &b) {
        std::vector<Lit> xs;
        for (size_t i = 0; i < a.size(); ++i) xs.push_back(neg(xor2(a[i], b[i])));
        return and_n(xs);
    }
    Lit ult(const Bits &a, const Bits &b) {      // unsigned a < b
        Lit lt = F;
        for (size_t i = 0; i < a.size(); ++i) {
            // from the LSB up: a < b on bits [0, i]
            Lit d = xor2(a[i], b[i]);
            lt = mux(d, b[i], lt);
        }
        return lt;
    }
    Lit slt(const Bits &a, const Bits &b) {
        Bits x = a, y = b;
        size_t m = a.size() - 1;
        x[m] = neg(x[m]);
        y[m] = neg(y[m]);
        return ult(x, y);
    }
    Bits ite(Lit c, const Bits &a, const Bits &b) {
        Bits r(a.size());
        for (size_t i = 0; i < a.size(); ++i) r[i] = mux(c, a[i], b[i]);
        return r;
    }
    bool all_const(const Bits &a) const {
        for (Lit l : a)
            if (!is_const(nrm(l))) return false;
        return true;
    }
    // a * b truncated to `outw` bits (operands zero-extended)
    Bits mul(const Bits &a0, const Bits &b0, size_t outw) {
        const Bits *a = &a0, *b = &b0;
        // put the constant (or the one with fewer non-false bits) on b
        auto weight = [&](const Bits &x) {
            size_t n = 0;
            for (Lit l : x) n += (nrm(l) != F);
            return n;
        };
        if (all_const(*a) && !all_const(*b)) std::swap(a, b);
        else if (!all_const(*b) && weight(*a) < weight(*b)) std::swap(a, b);
        Bits acc(outw, F);
        for (size_t i = 0; i < b->size() && i < outw; ++i) {
            Lit bi = nrm((*b)[i]);
            if (bi == F) continue;
            Bits row(outw, F);
            for (size_t j = 0; j + i < outw && j < a->size(); ++j) row[j + i] = and2((*a)[j], bi);
            // add only from bit i upward: the lower bits of row are false
            Lit c = F;
            for (size_t k = i; k < outw; ++k) {
                Lit s = xor2(xor2(acc[k], row[k]), c);
                c = maj(acc[k], row[k], c);
                acc[k] = s;
            }
        }
        return acc;
    }
    Bits zext(const Bits &a, size_t w) {
        Bits r = a;
        r.resize(w, F);
        return r;
    }
    // shifts by a word amount: SMT-LIB (>= width: 0 / sign fill)
    Bits shift(const Bits &a, const Bits &s, int kind) {      // 0 shl, 1 lshr, 2 ashr
        size_t w = a.size();
        Lit fill = kind == 2 ? a[w - 1] : F;
        Bits r = a;
        size_t k = 0;
        for (; k < s.size() && ((size_t)1 << k) < w; ++k) {
            size_t d = (size_t)1 << k;
            Bits t(w);
            for (size_t i = 0; i < w; ++i) {
                Lit moved;
                if (kind == 0) moved = i >= d ? r[i - d] : F;
                else moved = i + d < w ? r[i + d] : fill;
                t[i] = mux(s[k], moved, r[i]);
            }
            r = t;
        }
        // amount >= w: every bit is the fill
        std::vector<Lit> hi(s.begin() + (long)k, s.end());
        Lit big = or_n(hi);
        if (k < 64 && ((size_t)1 << k) > w) {
            // amounts in [w, 2^k) fit the low bits: compare them with w - 1
            Bits low(s.begin(), s.begin() + (long)k);
            Bits wm1(k);
            for (size_t i = 0; i < k; ++i) wm1[i] = (((w - 1) >> i) & 1u) ? T : F;
            big = or2(big, ult(wm1, low));
        }
        for (size_t i = 0; i < w; ++i) r[i] = mux(big, fill, r[i]);
        return r;
    }
};

// ---------------------------------------------------------------- blasting
struct ReadRec {
    uint32_t id;           // array or function id
    int kind;              // 1 array, 2 function
    std::vector<Bits> args;
    Bits val;
    uint32_t idx_node;     // an array read's index node (UINT32_MAX: none / a function)
};

const uint32_t NO_BASE = 0xffffffffu;

// A term as base + constant (mod 2^width): base NO_BASE for a constant.
struct Affine {
    uint32_t base;
    std::vector<uint32_t> off;
};

struct VecHash {
    size_t operator()(const std::vector<Lit> &v) const {
        uint64_t h = 1469598103934665603ull;
        for (Lit l : v) h = (h ^ (uint32_t)l) * 1099511628211ull;
        return (size_t)h;
    }
};

class Blaster {
public:
    // the node table, owned: a session appends to it query after query
    std::vector<uint32_t> nodes_, args_, limbs_;
    uint32_t n_nodes = 0, n_vars = 0;
    Sat S;
    Gates G;
    std::vector<Bits> memo;           // per node (1-bit nodes: size 1)
    std::vector<char> done;
    std::vector<Bits> var_bits;       // per variable id
    std::vector<uint32_t> var_width;
    std::vector<ReadRec> reads;
    // (array id / function id, kind, argument bits) -> read index
    std::unordered_map<std::vector<Lit>, size_t, VecHash> read_index;
    // (node, index bits) -> select result
    std::unordered_map<std::vector<Lit>, Bits, VecHash> select_memo;
    std::unordered_map<uint64_t, std::pair<Bits, Bits>> divmod_memo;
    std::vector<Affine> aff;
    std::vector<char> aff_done;
    bool bad = false;

    Blaster() : G(S) { limbs_.push_back(0u); }

    // Append a query's new nodes (their arguments are indices into the whole
    // table, their first_arg / constant limbs local to the query's arrays).
    bool append(const ms_query &q) {
        const uint32_t base = n_nodes;
        for (uint32_t k = 0; k < q.n_nodes; ++k) {
            const uint32_t *n = q.nodes + 6 * (size_t)k;
            if (n[0] >= MS_N_OPS) return false;
            uint32_t row[6] = {n[0], n[1], n[2], (uint32_t)args_.size(), n[4], n[5]};
            for (uint32_t i = 0; i < n[2]; ++i) {
                uint32_t a = q.args[n[3] + i];
                if (a >= base + k) return false;                     // post order
                args_.push_back(a);
            }
            if (n[0] == MS_CONST) {
                row[4] = (uint32_t)limbs_.size();
                limbs_.insert(limbs_.end(), q.limbs + n[4], q.limbs + n[4] + (n[1] + 31) / 32);
            }
            if (n[0] == MS_VAR && n[4] >= q.n_vars) return false;
            nodes_.insert(nodes_.end(), row, row + 6);
        }
        n_nodes = base + q.n_nodes;
        if (q.n_vars > n_vars) {
            n_vars = q.n_vars;
            var_bits.resize(n_vars);
            var_width.resize(n_vars, 0);
        }
        memo.resize(n_nodes);
        done.resize(n_nodes, 0);
        aff.resize(n_nodes);
        aff_done.resize(n_nodes, 0);
        return true;
    }

    // Word-level index reasoning: calldata and memory reads at `p + k` for one
    // symbolic p and many constants k (a CALLDATACOPY from a symbolic offset)
    // are pairwise distinct whenever their constants differ, so their Ackermann
    // pairs and store-chain hits are decided without an equality circuit.
    static void add_limbs(std::vector<uint32_t> &a, const std::vector<uint32_t> &b, uint32_t w, bool sub) {
        uint64_t carry = sub ? 1u : 0u;
        for (size_t i = 0; i < a.size(); ++i) {
            uint64_t x = (uint64_t)a[i] + (uint64_t)(sub ? ~b[i] : b[i]) + carry;
            a[i] = (uint32_t)x;
            carry = x >> 32;
        }
        if (w & 31u) a.back() &= (1u << (w & 31u)) - 1u;
    }
    const Affine &affine(uint32_t k) {
        if (aff_done[k]) return aff[k];
        const uint32_t *n = node(k);
        uint32_t w = n[1];
        size_t nl = (w + 31) / 32;
        Affine r{k, std::vector<uint32_t>(nl, 0u)};
        if (n[0] == MS_CONST) {
            r.base = NO_BASE;
            for (size_t i = 0; i < nl; ++i) r.off[i] = limbs_[n[4] + i];
        } else if ((n[0] == MS_BVADD || n[0] == MS_BVSUB) && n[2] == 2) {
            Affine a = affine(arg(k, 0));
            const Affine &b = affine(arg(k, 1));
            if (b.base == NO_BASE && a.off.size() == nl) {
                add_limbs(a.off, b.off, w, n[0] == MS_BVSUB);
                r = a;
            } else if (n[0] == MS_BVADD && a.base == NO_BASE && b.off.size() == nl) {
                Affine c = b;
                add_limbs(c.off, a.off, w, false);
                r = c;
            }
        }
        aff[k] = r;
        aff_done[k] = 1;
        return aff[k];
    }
    // 1: the two terms are equal, -1: they differ, 0: not known
    int relate(uint32_t a, uint32_t b) {
        if (a == NO_BASE || b == NO_BASE) return 0;
        if (a == b) return 1;
        const Affine &x = affine(a), &y = affine(b);
        if (x.base != y.base || x.off.size() != y.off.size()) return 0;
        return x.off == y.off ? 1 : -1;
    }
    const uint32_t *node(uint32_t k) const { return nodes_.data() + 6 * (size_t)k; }
    uint32_t arg(uint32_t k, uint32_t i) const { return args_[node(k)[3] + i]; }

    const Bits &get(uint32_t k) {
        if (!done[k]) { bad = true; static Bits empty; return empty; }
        return memo[k];
    }

    // The read of a base array / function at `args`: a fresh word.  Ackermann's
    // congruence between reads (equal arguments -> equal values) is added on
    // demand (lemmas_for): all O(n^2) pairs up front dominated the CNF when a
    // copy from a symbolic calldata offset reads hundreds of bytes.
    Bits point(int kind, uint32_t id, const std::vector<Bits> &args, uint32_t width, uint32_t idx_node = NO_BASE) {
        std::vector<Lit> key{kind, (int)id};
        for (const Bits &a : args) {
            key.push_back((int)a.size());
            key.insert(key.end(), a.begin(), a.end());
        }
        auto it = read_index.find(key);
        if (it != read_index.end()) return reads[it->second].val;
        // a read at the same index term (word-level) is the same read
        if (idx_node != NO_BASE) {
            for (const ReadRec &r : reads)
                if (r.kind == kind && r.id == id && relate(r.idx_node, idx_node) == 1 && r.val.size() == width)
                    return r.val;
        }
        Bits v = G.fresh_word(width);
        read_index.emplace(key, reads.size());
        reads.push_back({id, kind, args, v, idx_node});
        return v;
    }

    // Congruence lemmas the model violates: reads of one array / function with
    // equal argument values and different results get "args equal -> values
    // equal".  Returns the number added (0: the model is consistent).
    size_t lemmas_for(const std::vector<int8_t> &model) {
        auto val = [&](const Bits &b) {
            std::vector<uint32_t> out((b.size() + 31) / 32 + 1, 0u);
            out[0] = (uint32_t)b.size();
            for (size_t i = 0; i < b.size(); ++i) {
                Lit l = G.nrm(b[i]);
                bool v = l == G.T ? true : l == G.F ? false
                                                   : ((model[var(l)] == LU ? false : (bool)model[var(l)]) != sgn(l));
                if (v) out[1 + (i >> 5)] |= 1u << (i & 31);
            }
            return out;
        };
        auto assigned = [&](const Bits &b) {
            for (Lit l : b) {
                Lit n = G.nrm(l);
                if (n != G.T && n != G.F && model[var(n)] == LU) return false;
            }
            return true;
        };
        std::unordered_map<std::vector<Lit>, std::vector<size_t>, VecHash> groups;
        for (size_t i = 0; i < reads.size(); ++i) {
            // a read of another query's terms the search left unassigned has no
            // value to compare (its inputs are free: any extension can avoid or
            // match the others)
            bool full = assigned(reads[i].val);
            for (const Bits &a : reads[i].args) full = full && assigned(a);
            if (!full) continue;
            std::vector<Lit> key{reads[i].kind, (int)reads[i].id};
            for (const Bits &a : reads[i].args) {
                auto v = val(a);
                key.insert(key.end(), v.begin(), v.end());
            }
            groups[key].push_back(i);
        }
        size_t added = 0;
        for (auto &g : groups) {
            const std::vector<size_t> &ix = g.second;
            if (ix.size() < 2) continue;
            // chain every member to the first: a star of lemmas covers the group
            for (size_t m = 1; m < ix.size(); ++m) {
                size_t a = ix[0], b = ix[m];
                if (val(reads[a].val) == val(reads[b].val)) continue;
                if (congruence(a, b)) ++added;
            }
        }
        return added;
    }
    std::unordered_set<uint64_t> lemma_seen;
    size_t lemma_rounds = 0, lemmas = 0;

    // "args(a) == args(b) -> val(a) == val(b)" for reads a and b, once per pair
    bool congruence(size_t a, size_t b) {
        if (a > b) std::swap(a, b);
        uint64_t code = (uint64_t)a * 1000003ull + b;
        if (!lemma_seen.insert(code).second) return false;
        const ReadRec &r = reads[a], &t = reads[b];
        if (r.args.size() != t.args.size() || r.val.size() != t.val.size()) return false;
        std::vector<Lit> same;
        for (size_t i = 0; i < r.args.size(); ++i) {
            if (r.args[i].size() != t.args[i].size()) return false;
            same.push_back(G.eq(r.args[i], t.args[i]));
        }
        Lit all = G.and_n(same);
        for (size_t bit = 0; bit < r.val.size(); ++bit) {
            S.add_clause({neg(all), neg(r.val[bit]), t.val[bit]});
            S.add_clause({neg(all), r.val[bit], neg(t.val[bit])});
        }
        return true;
    }

    // Eager congruence for small-domain reads: a read whose arguments keep at
    // most EAGER_FREE free bits after level-0 folding gets its lemma against
    // every read of the same array / function at constant arguments its fixed
    // bits allow, before the search -- a Power(256, i % 32) application against
    // the 32 pinned points of the exponent table, say.  Lazily, the search first
    // picks a divisor that is no power of 256 and meets the table lemma by
    // lemma, each round a full re-solve (flag_array's division queries ran out
    // of budget that way).  Reads at wide symbolic arguments stay lazy.
    static constexpr size_t EAGER_FREE = 8;
    size_t eager_done = 0, eager_lemmas_added = 0;
    void eager_lemmas() {
        const size_t n = reads.size();
        if (eager_done == n) return;
        std::vector<int> freeb(n);
        for (size_t i = 0; i < n; ++i) {
            size_t f = 0;
            for (const Bits &a : reads[i].args)
                for (Lit l : a) {
                    Lit m = G.nrm(l);
                    if (m != G.T && m != G.F) ++f;
                }
            freeb[i] = (int)f;
        }
        auto compatible = [&](const ReadRec &x, const ReadRec &c) {
            if (x.args.size() != c.args.size()) return false;
            for (size_t i = 0; i < x.args.size(); ++i) {
                if (x.args[i].size() != c.args[i].size()) return false;
                for (size_t j = 0; j < x.args[i].size(); ++j) {
                    Lit s = G.nrm(x.args[i][j]), k = G.nrm(c.args[i][j]);
                    if ((s == G.T && k == G.F) || (s == G.F && k == G.T)) return false;
                }
            }
            return true;
        };
        for (size_t i = 0; i < n; ++i) {
            if (freeb[i] == 0 || (size_t)freeb[i] > EAGER_FREE) continue;
            for (size_t j = 0; j < n; ++j) {
                if (freeb[j] != 0 || (i < eager_done && j < eager_done)) continue;
                const ReadRec &x = reads[i], &c = reads[j];
                if (x.kind != c.kind || x.id != c.id || x.val.size() != c.val.size() || !compatible(x, c)) continue;
                if (congruence(i, j)) ++eager_lemmas_added;
            }
        }
        eager_done = n;
    }

    // solve with congruence lemmas on demand: LT only for a consistent model.
    // One conflict budget across the lemma rounds (0: unbounded).
    int8_t solve_lazy(const std::vector<Lit> &assume, uint64_t max_conflicts,
                      std::chrono::steady_clock::time_point deadline, bool timed) {
        const uint64_t c0 = S.conflicts;
        for (;;) {
            uint64_t left = 0;
            if (max_conflicts) {
                uint64_t used = S.conflicts - c0;
                if (used >= max_conflicts) return LU;
                left = max_conflicts - used;
            }
            int8_t r = S.solve(assume, left, deadline, timed);
            ++lemma_rounds;
            if (r != LT) return r;
            size_t got = lemmas_for(S.model);
            lemmas += got;
            if (got == 0) return LT;
            if (timed && std::chrono::steady_clock::now() > deadline) return LU;
        }
    }

    // select(array node k, index bits)
    Bits select(uint32_t k, const Bits &idx, uint32_t width, uint32_t idx_node) {
        std::vector<Lit> key{(int)k};
        key.insert(key.end(), idx.begin(), idx.end());
        auto it = select_memo.find(key);
        if (it != select_memo.end()) return it->second;
        const uint32_t *n = node(k);
        Bits r;
        if (n[0] == MS_K) {
            r = get(arg(k, 0));
        } else if (n[0] == MS_ARRAY) {
            r = point(1, n[4], {idx}, width, idx_node);
        } else if (n[0] == MS_STORE) {
            const Bits &i2 = get(arg(k, 1));
            const Bits &v = get(arg(k, 2));
            int rel = relate(arg(k, 1), idx_node);
            Lit hit = rel == 1 ? G.T : rel == -1 ? G.F : G.eq(i2, idx);
            if (hit == G.T) r = v;
            else if (hit == G.F) r = select(arg(k, 0), idx, width, idx_node);
            else {
                Bits rest = select(arg(k, 0), idx, width, idx_node);
                r = G.ite(hit, v, rest);
            }
        } else {
            bad = true;
            r = Bits(width, G.F);
        }
        select_memo.emplace(key, r);
        return r;
    }

    std::pair<Bits, Bits> udivrem(const Bits &a, const Bits &b, uint32_t ka, uint32_t kb) {
        uint64_t mk_ = ((uint64_t)ka << 32) | kb;
        auto it = divmod_memo.find(mk_);
        if (it != divmod_memo.end()) return it->second;
        size_t w = a.size();
        std::pair<Bits, Bits> out;
        if (G.all_const(b)) {
            // constant divisor: zero, a power of two, or any other
            int ones = 0, pos = -1;
            for (size_t i = 0; i < w; ++i)
                if (G.nrm(b[i]) == G.T) { ++ones; pos = (int)i; }
            if (ones == 0) {
                out = {Bits(w, G.T), a};
            } else if (ones == 1) {
                Bits qv(w, G.F), r(w, G.F);
                for (size_t i = 0; i + pos < w; ++i) qv[i] = a[i + pos];
                for (int i = 0; i < pos; ++i) r[i] = a[i];
                out = {qv, r};
            }
        }
        if (out.first.empty()) {
            // a divisor that is a read with a small-domain argument, pinned at
            // constant arguments to zero or powers of two (Power(256, i % 32)):
            // per pinned case the quotient is a shift, and the general divider
            // below only has to hold when no case applies
            std::vector<std::pair<Lit, int>> cases;   // (args equal, bit of the power; -1: zero)
            bool complete = false;
            const char *dc = std::getenv("MYTHSMT_DIVCASES");   // "0": general divider only (the A/B)
            Lit none = !(dc && dc[0] == '0') && divisor_cases(b, cases, complete) ? G.F : G.T;
            if (none == G.F && !complete) {
                std::vector<Lit> conds;
                for (auto &c : cases) conds.push_back(c.first);
                none = neg(G.or_n(conds));
            }
            // cases covering every value of the argument's free bits: exactly one
            // applies, and the general divider is never needed (none stays false)
            Bits qv = complete ? Bits(w, G.F) : G.fresh_word((uint32_t)w);
            Bits r = complete ? Bits(w, G.F) : G.fresh_word((uint32_t)w);
            if (!complete) {
                std::vector<Lit> zs;
                for (Lit l : b) zs.push_back(neg(l));
                Lit bz = G.and_n(zs);                     // b == 0
                // b != 0: a = q * b + r (in 2w bits, no wrap), r < b
                Bits prod = G.mul(G.zext(qv, 2 * w), G.zext(b, 2 * w), 2 * w);
                Bits sum = G.add(prod, G.zext(r, 2 * w), G.F);
                Lit ok1 = G.eq(sum, G.zext(a, 2 * w));
                Lit ok2 = G.ult(r, b);
                S.add_clause({neg(none), bz, ok1});
                S.add_clause({neg(none), bz, ok2});
                // b == 0: q = all ones, r = a (SMT-LIB)
                for (size_t i = 0; i < w; ++i) {
                    S.add_clause({neg(none), neg(bz), qv[i]});
                    S.add_clause({neg(none), neg(bz), neg(r[i]), a[i]});
                    S.add_clause({neg(none), neg(bz), r[i], neg(a[i])});
                }
            }
            for (auto &c : cases) {
                Bits cq(w, G.F), cr(w, G.F);
                if (c.second < 0) {
                    cq = Bits(w, G.T);
                    cr = a;
                } else {
                    size_t pos = (size_t)c.second;
                    for (size_t i = 0; i + pos < w; ++i) cq[i] = a[i + pos];
                    for (size_t i = 0; i < pos; ++i) cr[i] = a[i];
                }
                qv = G.ite(c.first, cq, qv);
                r = G.ite(c.first, cr, r);
            }
            out = {qv, r};
        }
        divmod_memo.emplace(mk_, out);
        return out;
    }

    // The pinned cases of a divisor (see udivrem): b is the value of a read
    // whose arguments keep at most EAGER_FREE free bits, and reads of the same
    // function / array at constant arguments its fixed bits allow have
    // constant values, each zero or a power of two.  Fills (args equal, bit)
    // per such read; false when b is no such read.  A case's value reaches b
    // through the congruence lemma of the pair (eager_lemmas, or lazily).
    bool divisor_cases(const Bits &b, std::vector<std::pair<Lit, int>> &cases, bool &complete) {
        const ReadRec *R = nullptr;
        for (const ReadRec &x : reads)
            if (x.val == b) { R = &x; break; }
        if (!R || R->args.empty()) {
            if (std::getenv("MYTHSMT_VERBOSE")) std::fprintf(stderr, "divisor_cases: divisor is no read\n");
            return false;
        }
        size_t fr = 0;
        for (const Bits &a : R->args)
            for (Lit l : a) {
                Lit m = G.nrm(l);
                if (m != G.T && m != G.F) ++fr;
            }
        if (fr == 0 || fr > EAGER_FREE) return false;
        complete = false;
        std::unordered_set<uint32_t> seen;          // the free bits' values the cases cover
        for (const ReadRec &c : reads) {
            if (&c == R || c.kind != R->kind || c.id != R->id || c.val.size() != b.size() ||
                c.args.size() != R->args.size())
                continue;
            bool cst = true, ok = true;
            for (size_t i = 0; i < c.args.size() && cst && ok; ++i) {
                if (c.args[i].size() != R->args[i].size()) { ok = false; break; }
                for (size_t j = 0; j < c.args[i].size(); ++j) {
                    Lit k = G.nrm(c.args[i][j]), s = G.nrm(R->args[i][j]);
                    if (k != G.T && k != G.F) { cst = false; break; }
                    if ((s == G.T && k == G.F) || (s == G.F && k == G.T)) { ok = false; break; }
                }
            }
            if (!cst || !ok) continue;
            int ones = 0, pos = -1;
            for (size_t i = 0; i < c.val.size(); ++i) {
                Lit v = G.nrm(c.val[i]);
                if (v != G.T && v != G.F) { ones = -1; break; }
                if (v == G.T) { ++ones; pos = (int)i; }
            }
            if (ones < 0 || ones > 1) continue;         // not pinned / no power of two: the general case
            std::vector<Lit> same;
            for (size_t i = 0; i < c.args.size(); ++i) same.push_back(G.eq(R->args[i], c.args[i]));
            cases.push_back({G.and_n(same), ones == 0 ? -1 : pos});
            uint32_t key = 0, at = 0;
            for (size_t i = 0; i < c.args.size(); ++i)
                for (size_t j = 0; j < c.args[i].size(); ++j) {
                    Lit sr = G.nrm(R->args[i][j]);
                    if (sr == G.T || sr == G.F) continue;
                    if (G.nrm(c.args[i][j]) == G.T) key |= 1u << at;
                    ++at;
                }
            seen.insert(key);
        }
        // every value of the free bits has its case: no general divider needed
        complete = seen.size() == (size_t)1 << fr;
        if (std::getenv("MYTHSMT_VERBOSE")) std::fprintf(stderr, "divisor_cases: %zu cases, %zu free bits\n", cases.size(), fr);
        return !cases.empty();
    }

    Bits absv(const Bits &a) { return G.ite(a.back(), G.bneg(a), a); }

    void blast(uint32_t k) {
        const uint32_t *n = node(k);
        const uint32_t op = n[0], w = n[1], na = n[2];
        Bits r;
        auto A = [&](uint32_t i) -> const Bits & { return get(arg(k, i)); };
        auto bit = [&](Lit l) { return Bits{l}; };
        switch (op) {
        case MS_CONST: r = G.cnst(w, limbs_.data() + n[4]); break;
        case MS_VAR: {
            uint32_t id = n[4];
            if (id >= n_vars) { bad = true; return; }
            if (var_bits[id].empty()) { var_bits[id] = G.fresh_word(w); var_width[id] = w; }
            if (var_bits[id].size() != w) { bad = true; return; }
            r = var_bits[id];
            break;
        }
        case MS_BVADD: r = G.add(A(0), A(1), G.F); break;
        case MS_BVSUB: r = G.sub(A(0), A(1)); break;
        case MS_BVMUL: r = G.mul(A(0), A(1), w); break;
        case MS_BVUDIV: r = udivrem(A(0), A(1), arg(k, 0), arg(k, 1)).first; break;
        case MS_BVUREM: r = udivrem(A(0), A(1), arg(k, 0), arg(k, 1)).second; break;
        case MS_BVSDIV: case MS_BVSREM: case MS_BVSMOD: {
            const Bits &a = A(0), &b = A(1);
            Lit sa = a.back(), sb = b.back();
            // |a|, |b| as fresh-keyed words: memo on the operand nodes with the op
            Bits ua = absv(a), ub = absv(b);
            auto dr = udivrem(ua, ub, 0x80000000u | k, 0x80000000u | op);
            if (op == MS_BVSDIV) {
                r = G.ite(G.xor2(sa, sb), G.bneg(dr.first), dr.first);
            } else if (op == MS_BVSREM) {
                r = G.ite(sa, G.bneg(dr.second), dr.second);
            } else {
                const Bits &u = dr.second;
                std::vector<Lit> zs;
                for (Lit l : u) zs.push_back(neg(l));
                Lit uz = G.and_n(zs);
                Bits negu = G.bneg(u);
                Bits t1 = G.add(negu, b, G.F);      // s < 0, t >= 0
                Bits t2 = G.add(u, b, G.F);         // s >= 0, t < 0
                Bits m = G.ite(sa, G.ite(sb, negu, t1), G.ite(sb, t2, u));
                r = G.ite(uz, u, m);
            }
            break;
        }
        case MS_BVAND: case MS_BVOR: case MS_BVXOR: {
            const Bits &a = A(0), &b = A(1);
            r.resize(w);
            for (uint32_t i = 0; i < w; ++i)
                r[i] = op == MS_BVAND ? G.and2(a[i], b[i]) : op == MS_BVOR ? G.or2(a[i], b[i]) : G.xor2(a[i], b[i]);
            break;
        }
        case MS_BVNOT: r = G.bnot(A(0)); break;
        case MS_BVNEG: r = G.bneg(A(0)); break;
        case MS_BVSHL: r = G.shift(A(0), A(1), 0); break;
        case MS_BVLSHR: r = G.shift(A(0), A(1), 1); break;
        case MS_BVASHR: r = G.shift(A(0), A(1), 2); break;
        case MS_EQ: r = bit(G.eq(A(0), A(1))); break;
        case MS_DISTINCT: r = bit(neg(G.eq(A(0), A(1)))); break;
        case MS_BVULT: r = bit(G.ult(A(0), A(1))); break;
        case MS_BVULE: r = bit(neg(G.ult(A(1), A(0)))); break;
        case MS_BVUGT: r = bit(G.ult(A(1), A(0))); break;
        case MS_BVUGE: r = bit(neg(G.ult(A(0), A(1)))); break;
        case MS_BVSLT: r = bit(G.slt(A(0), A(1))); break;
        case MS_BVSLE: r = bit(neg(G.slt(A(1), A(0)))); break;
        case MS_BVSGT: r = bit(G.slt(A(1), A(0))); break;
        case MS_BVSGE: r = bit(neg(G.slt(A(0), A(1)))); break;
        case MS_AND: case MS_OR: {
            std::vector<Lit> xs;
            for (uint32_t i = 0; i < na; ++i) xs.push_back(A(i)[0]);
            r = bit(op == MS_AND ? G.and_n(xs) : G.or_n(xs));
            break;
        }
        case MS_NOT: r = bit(neg(A(0)[0])); break;
        case MS_XOR: r = bit(G.xor2(A(0)[0], A(1)[0])); break;
        case MS_IMPLIES: r = bit(G.or2(neg(A(0)[0]), A(1)[0])); break;
        case MS_ITE: r = G.ite(A(0)[0], A(1), A(2)); break;
        case MS_CONCAT: {
            const Bits &hi = A(0), &lo = A(1);
            r = lo;
            r.insert(r.end(), hi.begin(), hi.end());
            break;
        }
        case MS_EXTRACT: {
            const Bits &a = A(0);
            uint32_t hi = n[4], lo = n[5];
            if (hi >= a.size() || lo > hi) { bad = true; return; }
            r.assign(a.begin() + lo, a.begin() + hi + 1);
            break;
        }
        case MS_ZERO_EXTEND: r = G.zext(A(0), w); break;
        case MS_SIGN_EXTEND: {
            r = A(0);
            Lit s = r.back();
            r.resize(w, s);
            break;
        }
        case MS_BVADD_NOOVFL_U: {
            Lit c;
            G.add(A(0), A(1), G.F, &c);
            r = bit(neg(c));
            break;
        }
        case MS_BVUMUL_NOOVFL: {
            size_t wa = A(0).size();
            Bits p = G.mul(G.zext(A(0), 2 * wa), G.zext(A(1), 2 * wa), 2 * wa);
            std::vector<Lit> hi(p.begin() + (long)wa, p.end());
            r = bit(neg(G.or_n(hi)));
            break;
        }
        case MS_BVSUB_NOUDFL_U: r = bit(neg(G.ult(A(0), A(1)))); break;
        case MS_SELECT: r = select(arg(k, 0), A(1), w, arg(k, 1)); break;
        case MS_UF: {
            std::vector<Bits> as;
            for (uint32_t i = 0; i < na; ++i) as.push_back(A(i));
            r = point(2, n[4], as, w);
            break;
        }
        case MS_ARRAY: case MS_K: case MS_STORE: r.clear(); break;       // array-sorted: read through select
        default: bad = true; return;
        }
        if (op != MS_ARRAY && op != MS_K && op != MS_STORE && r.size() != (w ? w : r.size())) { bad = true; return; }
        memo[k] = std::move(r);
        done[k] = 1;
    }
};

void put_bits(std::vector<uint32_t> &out, const Bits &b, const std::vector<int8_t> &model, Lit T) {
    size_t nl = (b.size() + 31) / 32;
    size_t at = out.size();
    out.resize(at + nl, 0u);
    for (size_t i = 0; i < b.size(); ++i) {
        Lit l = b[i];
        bool v;
        if (l == T) v = true;
        else if (l == neg(T)) v = false;
        else {
            int8_t a = model[var(l)];
            v = (a == LU ? false : (bool)a) != sgn(l);
        }
        if (v) out[at + (i >> 5)] |= 1u << (i & 31);
    }
}

}  // namespace

extern "C" int ms_abi_version(void) { return MS_ABI_VERSION; }

namespace {

// Blast the query's conjuncts (each asserted as it is built when `units`, the
// stateless call; as assumptions in a session, whose clause database must stay
// true of every later query), solve with congruence lemmas on demand,
// minimise, write the model stream.
int run(Blaster &B, const ms_query *q, const ms_limits *lim, bool units, uint32_t *model, uint32_t model_cap,
        uint32_t *model_len, ms_stats *stats) {
    auto t0 = std::chrono::steady_clock::now();
    const uint32_t max_ms = lim ? lim->max_ms : 0u;
    const uint64_t max_conf = lim ? lim->max_conflicts : 0u;
    auto deadline = t0 + std::chrono::milliseconds(max_ms);
    const uint64_t conf0 = B.S.conflicts, dec0 = B.S.decisions, prop0 = B.S.propagations;
    if (!B.append(*q)) return MS_EINVAL;
    for (uint32_t i = 0; i < q->n_roots; ++i)
        if (q->roots[i] >= B.n_nodes || B.node(q->roots[i])[1] != 1) return MS_EINVAL;
    for (uint32_t i = 0; i < q->n_minimize; ++i)
        if (q->minimize[i] >= B.n_nodes) return MS_EINVAL;
    // Each conjunct is blasted (and, stateless, asserted) in turn, the smaller
    // cones first: a bound (cnt <= 20), an equality with a constant, a selector
    // check fixes bits at level 0 before the multipliers, store chains and
    // congruence lemmas that read them are built, and those gates fold
    // (Gates::nrm) instead of entering the CNF.
    std::vector<uint32_t> order(q->roots, q->roots + q->n_roots);
    std::stable_sort(order.begin(), order.end());
    uint32_t blasted = 0;
    bool timed_out = false;
    auto cone = [&](uint32_t root) {
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        while (!st.empty() && !B.bad) {
            auto [k, ready] = st.back();
            st.pop_back();
            if (B.done[k]) continue;
            if (!ready) {
                st.push_back({k, true});
                const uint32_t *n = B.node(k);
                for (uint32_t i = n[2]; i-- > 0;)
                    if (!B.done[B.arg(k, i)]) st.push_back({B.arg(k, i), false});
                continue;
            }
            size_t first_input = B.G.inputs.size();
            B.blast(k);
            // decide the words' bits first: every gate output follows from them
            // by propagation (the Tseitin encodings are complete), so the search
            // does not wander through the gate variables
            for (size_t j = first_input; j < B.G.inputs.size(); ++j) {
                int v = B.G.inputs[j];
                B.S.activity[v] = std::max(B.S.activity[v], B.S.var_inc);
                if (B.S.heap_pos[v] >= 0) B.S.heap_up(B.S.heap_pos[v]);
            }
            if (max_ms && (++blasted & 63u) == 0 && std::chrono::steady_clock::now() > deadline) {
                timed_out = true;
                return;
            }
        }
    };
    std::vector<Lit> assume;
    for (uint32_t r : order) {
        cone(r);
        if (B.bad) return MS_EINVAL;
        if (timed_out) break;
        if (B.memo[r].size() != 1) return MS_EINVAL;
        if (units) {
            B.S.add_clause({B.memo[r][0]});
            if (!B.S.ok) break;                        // a conflict at level 0: unsat
        } else {
            assume.push_back(B.memo[r][0]);
        }
    }
    for (uint32_t i = 0; i < q->n_minimize && B.S.ok && !timed_out; ++i) {
        cone(q->minimize[i]);
        if (B.bad) return MS_EINVAL;
    }
    {
        const char *eager = std::getenv("MYTHSMT_EAGER");       // "0": lazy only (the A/B)
        if (B.S.ok && !timed_out && !(eager && eager[0] == '0')) B.eager_lemmas();
    }
    auto fill_stats = [&](uint32_t solves) {
        if (!stats) return;
        stats->vars = (uint64_t)B.S.n_vars();
        stats->clauses = B.S.n_clauses;
        stats->conflicts = B.S.conflicts - conf0;
        stats->decisions = B.S.decisions - dec0;
        stats->propagations = B.S.propagations - prop0;
        stats->solves = solves;
        stats->ms = (uint32_t)std::chrono::duration_cast<std::chrono::milliseconds>(
            std::chrono::steady_clock::now() - t0).count();
    };
    if (timed_out) {
        fill_stats(0);
        return MS_UNKNOWN;
    }
    // the model of this query: the variables, arrays and functions its cone
    // mentions (a session holds others, of earlier queries)
    std::vector<char> in_cone(B.n_nodes, 0), var_in(B.n_vars, 0);
    std::unordered_set<uint64_t> tables;          // (kind << 32) | id
    {
        std::vector<uint32_t> st(q->roots, q->roots + q->n_roots);
        st.insert(st.end(), q->minimize, q->minimize + q->n_minimize);
        while (!st.empty()) {
            uint32_t k = st.back();
            st.pop_back();
            if (in_cone[k]) continue;
            in_cone[k] = 1;
            const uint32_t *n = B.node(k);
            if (n[0] == MS_VAR) var_in[n[4]] = 1;
            else if (n[0] == MS_ARRAY) tables.insert((1ull << 32) | n[4]);
            else if (n[0] == MS_UF) tables.insert((2ull << 32) | n[4]);
            for (uint32_t i = 0; i < n[2]; ++i) st.push_back(B.arg(k, i));
        }
    }
    // A session query is first decided over its own cone's inputs only
    // (Sat::set_relevant) on a small conflict budget: a satisfiable query then
    // leaves the other queries' variables unassigned instead of deciding the
    // whole session (2.5x faster on exceptions.sol.o).  A query that needs
    // more than 20 conflicts goes on over every variable with the full budget:
    // restricted decisions cost ~7x more per conflict on BECToken's
    // multiplications (profiles/r06/exact_budget.txt).  MYTHSMT_REL_BUDGET sets the first
    // budget (0: off); MYTHSMT_RELEVANT=1 keeps the restriction for the whole
    // budget (the A/B).
    std::vector<int> relevant;
    const char *rel_env = std::getenv("MYTHSMT_REL_BUDGET");
    const bool rel_only = std::getenv("MYTHSMT_RELEVANT") != nullptr;
    const uint64_t rel_budget = rel_only ? max_conf : rel_env ? std::strtoull(rel_env, nullptr, 10) : 20u;
    const bool use_rel = !units && (rel_only || rel_budget > 0);
    if (use_rel) {
        auto add_bits = [&](const Bits &b) {
            for (Lit l : b)
                if (l != B.G.T && l != B.G.F) relevant.push_back(var(l));
        };
        for (uint32_t v = 0; v < B.n_vars; ++v)
            if (var_in[v]) add_bits(B.var_bits[v]);
        for (const ReadRec &r : B.reads)
            if (tables.count(((uint64_t)r.kind << 32) | r.id)) add_bits(r.val);
        for (uint32_t k = 0; k < B.n_nodes; ++k) {
            if (!in_cone[k]) continue;
            const uint32_t *n = B.node(k);
            uint64_t key;
            if (n[0] == MS_BVUDIV || n[0] == MS_BVUREM) key = ((uint64_t)B.arg(k, 0) << 32) | B.arg(k, 1);
            else if (n[0] == MS_BVSDIV || n[0] == MS_BVSREM || n[0] == MS_BVSMOD)
                key = ((uint64_t)(0x80000000u | k) << 32) | (0x80000000u | n[0]);
            else continue;
            auto it = B.divmod_memo.find(key);
            if (it != B.divmod_memo.end()) {
                add_bits(it->second.first);
                add_bits(it->second.second);
            }
        }
        std::sort(relevant.begin(), relevant.end());
        relevant.erase(std::unique(relevant.begin(), relevant.end()), relevant.end());
    }
    auto t_blast = std::chrono::steady_clock::now();
    int8_t res;
    if (use_rel) {
        B.S.set_relevant(&relevant);
        res = B.solve_lazy(assume, rel_budget, deadline, max_ms != 0);
        B.S.set_relevant(nullptr);                    // every variable again
        bool late = max_ms != 0 && std::chrono::steady_clock::now() > deadline;
        if (res == LU && !rel_only && !late)
            res = B.solve_lazy(assume, max_conf, deadline, max_ms != 0);
    } else {
        res = B.solve_lazy(assume, max_conf, deadline, max_ms != 0);
    }
    if (std::getenv("MYTHSMT_VERBOSE"))
        std::fprintf(stderr, "ms_solve: blast %.1f ms (%d vars, %llu clauses, %zu reads), solve %.1f ms, %llu conflicts, "
                             "%zu rounds, %zu lemmas, %llu decisions\n",
                     std::chrono::duration<double, std::milli>(t_blast - t0).count(), B.S.n_vars(),
                     (unsigned long long)B.S.n_clauses, B.reads.size(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_blast).count(),
                     (unsigned long long)(B.S.conflicts - conf0), B.lemma_rounds, B.lemmas,
                     (unsigned long long)(B.S.decisions - dec0));
    uint32_t solves = 1;
    std::vector<int8_t> best = B.S.model;
    if (res == LT && q->n_minimize) {
        // lexicographic minimisation (z3 Optimize's default priority), MSB
        // first under assumptions; the best model so far stands on budget
        // per bit a conflict budget (deterministic); the wall clock only guards
        auto mdeadline = std::chrono::steady_clock::now() +
                         std::chrono::milliseconds(lim && lim->minimize_ms ? lim->minimize_ms : 10000u);
        bool stop = false;
        for (uint32_t m = 0; m < q->n_minimize && !stop; ++m) {
            const Bits bits = B.memo[q->minimize[m]];
            for (size_t i = bits.size(); i-- > 0 && !stop;) {
                Lit l = B.G.nrm(bits[i]);
                if (l == B.G.T || l == B.G.F) continue;
                int8_t cur = best[var(l)];
                bool cur_v = (cur == LU ? false : (bool)cur) != sgn(l);
                assume.push_back(neg(l));
                if (!cur_v) continue;
                int8_t r2 = B.solve_lazy(assume, 20000, mdeadline, true);
                ++solves;
                if (r2 == LT) best = B.S.model;
                else {
                    assume.back() = l;
                    if (r2 == LU) stop = true;
                }
            }
        }
    }
    fill_stats(solves);
    if (res == LF) return MS_UNSAT;
    if (res == LU) return MS_UNKNOWN;
    std::vector<uint32_t> out;
    for (uint32_t v = 0; v < B.n_vars; ++v) {
        if (B.var_bits[v].empty() || !var_in[v]) continue;
        out.push_back(3u);
        out.push_back(v);
        put_bits(out, B.var_bits[v], best, B.G.T);
    }
    auto assigned = [&](const Bits &b) {
        for (Lit l : b) {
            Lit n = B.G.nrm(l);
            if (n != B.G.T && n != B.G.F && best[var(n)] == LU) return false;
        }
        return true;
    };
    for (const ReadRec &r : B.reads) {
        if (!tables.count(((uint64_t)r.kind << 32) | r.id)) continue;
        bool full = assigned(r.val);
        for (const Bits &a : r.args) full = full && assigned(a);
        if (!full) continue;                  // another query's read the search left open
        out.push_back((uint32_t)r.kind);
        out.push_back(r.id);
        for (const Bits &a : r.args) put_bits(out, a, best, B.G.T);
        put_bits(out, r.val, best, B.G.T);
    }
    out.push_back(0u);
    if (model_len) *model_len = (uint32_t)out.size();
    if (out.size() > model_cap || !model) return MS_ESPACE;
    std::memcpy(model, out.data(), out.size() * 4);
    return MS_SAT;
}

}  // namespace

struct ms_session {
    Blaster B;
};

extern "C" int ms_solve(const ms_query *q, const ms_limits *lim, uint32_t *model, uint32_t model_cap,
                        uint32_t *model_len, ms_stats *stats) {
    try {
        if (!q || (q->n_nodes && (!q->nodes || !q->args)) || (q->n_roots && !q->roots)) return MS_EINVAL;
        Blaster B;
        return run(B, q, lim, true, model, model_cap, model_len, stats);
    } catch (...) {
        return MS_EINVAL;
    }
}

extern "C" int ms_session_open(ms_session **out) {
    try {
        if (!out) return MS_EINVAL;
        *out = new ms_session();
        return 0;
    } catch (...) {
        return MS_EINVAL;
    }
}

extern "C" void ms_session_close(ms_session *s) { delete s; }

extern "C" int ms_session_solve(ms_session *s, const ms_query *q, const ms_limits *lim, uint32_t *model,
                                uint32_t model_cap, uint32_t *model_len, ms_stats *stats) {
    try {
        if (!s || !q || (q->n_nodes && (!q->nodes || !q->args)) || (q->n_roots && !q->roots)) return MS_EINVAL;
        return run(s->B, q, lim, false, model, model_cap, model_len, stats);
    } catch (...) {
        return MS_EINVAL;
    }
}
