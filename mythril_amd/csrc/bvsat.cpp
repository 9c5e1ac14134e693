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
#include <cstring>
#include <unordered_map>
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

    // Level-0 clause: simplified against the current level-0 assignment.
    bool add_clause(std::vector<Lit> ls) {
        if (!ok) return false;
        std::sort(ls.begin(), ls.end());
        std::vector<Lit> out;
        Lit prev = -1;
        for (Lit l : ls) {
            if (value(l) == LT || l == neg(prev)) return true;
            if (value(l) != LF && l != prev) out.push_back(l);
            prev = l;
        }
        ++n_clauses;
        if (out.empty()) return ok = false;
        if (out.size() == 1) {
            enqueue(out[0], CR_NONE);
            return ok = (propagate() == CR_NONE);
        }
        attach(alloc(out, false));
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
            heap_insert(v);
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
    Lit and2(Lit a, Lit b) {
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
    Bits fresh_word(uint32_t w) {
        Bits b(w);
        for (auto &x : b) x = fresh();
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
            if (!is_const(l)) return false;
        return true;
    }
    // a * b truncated to `outw` bits (operands zero-extended)
    Bits mul(const Bits &a0, const Bits &b0, size_t outw) {
        const Bits *a = &a0, *b = &b0;
        // put the constant (or the one with fewer non-false bits) on b
        auto weight = [&](const Bits &x) {
            size_t n = 0;
            for (Lit l : x) n += (l != F);
            return n;
        };
        if (all_const(*a) && !all_const(*b)) std::swap(a, b);
        else if (!all_const(*b) && weight(*a) < weight(*b)) std::swap(a, b);
        Bits acc(outw, F);
        for (size_t i = 0; i < b->size() && i < outw; ++i) {
            Lit bi = (*b)[i];
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
    const ms_query &q;
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
    bool bad = false;

    explicit Blaster(const ms_query &qq) : q(qq), G(S) {
        memo.resize(q.n_nodes);
        done.assign(q.n_nodes, 0);
        var_bits.resize(q.n_vars);
        var_width.assign(q.n_vars, 0);
    }
    const uint32_t *node(uint32_t k) const { return q.nodes + 6 * (size_t)k; }
    uint32_t arg(uint32_t k, uint32_t i) const { return q.args[node(k)[3] + i]; }

    const Bits &get(uint32_t k) {
        if (!done[k]) { bad = true; static Bits empty; return empty; }
        return memo[k];
    }

    // the read of a base array / function at `args`, Ackermannised against the
    // earlier reads of the same one
    Bits point(int kind, uint32_t id, const std::vector<Bits> &args, uint32_t width) {
        std::vector<Lit> key{kind, (int)id};
        for (const Bits &a : args) {
            key.push_back((int)a.size());
            key.insert(key.end(), a.begin(), a.end());
        }
        auto it = read_index.find(key);
        if (it != read_index.end()) return reads[it->second].val;
        Bits v = G.fresh_word(width);
        for (const ReadRec &r : reads) {
            if (r.kind != kind || r.id != id || r.args.size() != args.size()) continue;
            std::vector<Lit> same;
            bool width_ok = true;
            for (size_t i = 0; i < args.size(); ++i) {
                if (r.args[i].size() != args[i].size()) { width_ok = false; break; }
                same.push_back(G.eq(r.args[i], args[i]));
            }
            if (!width_ok || r.val.size() != width) continue;
            Lit all = G.and_n(same);
            if (all == G.F) continue;
            // all -> v == r.val, bit by bit
            for (size_t b = 0; b < width; ++b) {
                S.add_clause({neg(all), neg(v[b]), r.val[b]});
                S.add_clause({neg(all), v[b], neg(r.val[b])});
            }
        }
        read_index.emplace(key, reads.size());
        reads.push_back({id, kind, args, v});
        return v;
    }

    // select(array node k, index bits)
    Bits select(uint32_t k, const Bits &idx, uint32_t width) {
        std::vector<Lit> key{(int)k};
        key.insert(key.end(), idx.begin(), idx.end());
        auto it = select_memo.find(key);
        if (it != select_memo.end()) return it->second;
        const uint32_t *n = node(k);
        Bits r;
        if (n[0] == MS_K) {
            r = get(arg(k, 0));
        } else if (n[0] == MS_ARRAY) {
            r = point(1, n[4], {idx}, width);
        } else if (n[0] == MS_STORE) {
            const Bits &i2 = get(arg(k, 1));
            const Bits &v = get(arg(k, 2));
            Lit hit = G.eq(i2, idx);
            if (hit == G.T) r = v;
            else {
                Bits rest = select(arg(k, 0), idx, width);
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
                if (b[i] == G.T) { ++ones; pos = (int)i; }
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
            Bits qv = G.fresh_word((uint32_t)w), r = G.fresh_word((uint32_t)w);
            std::vector<Lit> zs;
            for (Lit l : b) zs.push_back(neg(l));
            Lit bz = G.and_n(zs);                     // b == 0
            // b != 0: a = q * b + r (in 2w bits, no wrap), r < b
            Bits prod = G.mul(G.zext(qv, 2 * w), G.zext(b, 2 * w), 2 * w);
            Bits sum = G.add(prod, G.zext(r, 2 * w), G.F);
            Lit ok1 = G.eq(sum, G.zext(a, 2 * w));
            Lit ok2 = G.ult(r, b);
            S.add_clause({bz, ok1});
            S.add_clause({bz, ok2});
            // b == 0: q = all ones, r = a (SMT-LIB)
            for (size_t i = 0; i < w; ++i) {
                S.add_clause({neg(bz), qv[i]});
                S.add_clause({neg(bz), neg(r[i]), a[i]});
                S.add_clause({neg(bz), r[i], neg(a[i])});
            }
            out = {qv, r};
        }
        divmod_memo.emplace(mk_, out);
        return out;
    }

    Bits absv(const Bits &a) { return G.ite(a.back(), G.bneg(a), a); }

    void blast(uint32_t k) {
        const uint32_t *n = node(k);
        const uint32_t op = n[0], w = n[1], na = n[2];
        Bits r;
        auto A = [&](uint32_t i) -> const Bits & { return get(arg(k, i)); };
        auto bit = [&](Lit l) { return Bits{l}; };
        switch (op) {
        case MS_CONST: r = G.cnst(w, q.limbs + n[4]); break;
        case MS_VAR: {
            uint32_t id = n[4];
            if (id >= q.n_vars) { bad = true; return; }
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
        case MS_SELECT: r = select(arg(k, 0), A(1), w); break;
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

extern "C" int ms_solve(const ms_query *q, const ms_limits *lim, uint32_t *model, uint32_t model_cap,
                        uint32_t *model_len, ms_stats *stats) {
    try {
        if (!q || !q->nodes || (q->n_roots && !q->roots)) return MS_EINVAL;
        auto t0 = std::chrono::steady_clock::now();
        const uint32_t max_ms = lim ? lim->max_ms : 0u;
        const uint64_t max_conf = lim ? lim->max_conflicts : 0u;
        auto deadline = t0 + std::chrono::milliseconds(max_ms);
        Blaster B(*q);
        for (uint32_t k = 0; k < q->n_nodes; ++k) {
            const uint32_t *n = B.node(k);
            if (n[0] >= MS_N_OPS) return MS_EINVAL;
            for (uint32_t i = 0; i < n[2]; ++i)
                if (B.arg(k, i) >= k) return MS_EINVAL;           // post order
            B.blast(k);
            if (B.bad) return MS_EINVAL;
            if (max_ms && (k & 63u) == 0 && std::chrono::steady_clock::now() > deadline) {
                if (stats) std::memset(stats, 0, sizeof(*stats));
                return MS_UNKNOWN;
            }
        }
        for (uint32_t i = 0; i < q->n_roots; ++i) {
            uint32_t r = q->roots[i];
            if (r >= q->n_nodes || B.memo[r].size() != 1) return MS_EINVAL;
            B.S.add_clause({B.memo[r][0]});
        }
        int8_t res = B.S.solve({}, max_conf, deadline, max_ms != 0);
        uint32_t solves = 1;
        std::vector<int8_t> best = B.S.model;
        if (res == LT && q->n_minimize) {
            // lexicographic minimisation (z3 Optimize's default priority), MSB
            // first under assumptions; the best model so far stands on budget
            auto mdeadline = std::chrono::steady_clock::now() +
                             std::chrono::milliseconds(lim && lim->minimize_ms ? lim->minimize_ms : 2000u);
            std::vector<Lit> assume;
            bool stop = false;
            for (uint32_t m = 0; m < q->n_minimize && !stop; ++m) {
                uint32_t k = q->minimize[m];
                if (k >= q->n_nodes) return MS_EINVAL;
                const Bits bits = B.memo[k];
                for (size_t i = bits.size(); i-- > 0 && !stop;) {
                    Lit l = bits[i];
                    if (l == B.G.T || l == B.G.F) continue;
                    int8_t cur = best[var(l)];
                    bool cur_v = (cur == LU ? false : (bool)cur) != sgn(l);
                    if (!cur_v) { assume.push_back(neg(l)); continue; }
                    assume.push_back(neg(l));
                    int8_t r2 = B.S.solve(assume, 20000, mdeadline, true);
                    ++solves;
                    if (r2 == LT) best = B.S.model;
                    else {
                        assume.back() = l;
                        if (r2 == LU) stop = true;
                    }
                }
            }
        }
        uint32_t ms = (uint32_t)std::chrono::duration_cast<std::chrono::milliseconds>(
            std::chrono::steady_clock::now() - t0).count();
        if (stats) {
            stats->vars = (uint64_t)B.S.n_vars();
            stats->clauses = B.S.n_clauses;
            stats->conflicts = B.S.conflicts;
            stats->decisions = B.S.decisions;
            stats->propagations = B.S.propagations;
            stats->solves = solves;
            stats->ms = ms;
        }
        if (res == LF) return MS_UNSAT;
        if (res == LU) return MS_UNKNOWN;
        std::vector<uint32_t> out;
        for (uint32_t v = 0; v < q->n_vars; ++v) {
            if (B.var_bits[v].empty()) {
                // a variable no node uses: its width is unknown here; 0 limbs
                continue;
            }
            put_bits(out, B.var_bits[v], best, B.G.T);
        }
        for (const ReadRec &r : B.reads) {
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
    } catch (...) {
        return MS_EINVAL;
    }
}
