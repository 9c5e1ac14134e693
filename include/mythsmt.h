/* mythsmt.h -- the exact bit-vector decision procedure behind kernel 2's prefilter.
 *
 * libmythsmt.so (host C++, mythril_amd/csrc/bvsat.cpp) decides the path-constraint
 * queries kernel 2's quick-sat and the SAT-only search leave open: it is the
 * counterpart of the reference's z3 `Optimize().check()` call in get_model
 * (mythril/support/model.py:37-82 -- sat with a model, unsat -> UnsatError,
 * timeout -> SolverTimeOutException) for the operator set mythril/laser/smt
 * emits (bitvec.py, bitvec_helper.py, bool.py, array.py, function.py) and
 * z3's `minimize` objectives (analysis/solver.py:219-259, lexicographic).
 * Decision: bit-blasting (Tseitin, structurally hashed gates), arrays by
 * store-chain expansion + Ackermann reads, uninterpreted functions (keccak256_N,
 * its inverse, Power) by Ackermann congruence, and a CDCL SAT core.
 *
 * Threading: one call is self-contained (no global state); calls may run on
 * several host threads at once.  Errors are negative return codes; no call
 * throws across the ABI.
 */
#ifndef MYTHSMT_H
#define MYTHSMT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MS_ABI_VERSION 1

/* node opcodes (mythril_amd/smt/expr.py op names) */
enum {
    MS_CONST = 0, MS_VAR, MS_BVADD, MS_BVSUB, MS_BVMUL, MS_BVUDIV, MS_BVUREM, MS_BVSDIV, MS_BVSREM, MS_BVSMOD,
    MS_BVAND, MS_BVOR, MS_BVXOR, MS_BVNOT, MS_BVNEG, MS_BVSHL, MS_BVLSHR, MS_BVASHR,
    MS_EQ, MS_DISTINCT, MS_BVULT, MS_BVULE, MS_BVUGT, MS_BVUGE, MS_BVSLT, MS_BVSLE, MS_BVSGT, MS_BVSGE,
    MS_AND, MS_OR, MS_NOT, MS_XOR, MS_IMPLIES, MS_ITE, MS_CONCAT, MS_EXTRACT, MS_ZERO_EXTEND, MS_SIGN_EXTEND,
    MS_BVADD_NOOVFL_U, MS_BVUMUL_NOOVFL, MS_BVSUB_NOUDFL_U, MS_SELECT, MS_UF, MS_ARRAY, MS_K, MS_STORE,
    MS_N_OPS
};

/* A query: nodes in post order (every argument before its user).
 * node k = nodes[6k .. 6k+5] = {op, width, n_args, first_arg, p0, p1}; its
 * arguments are args[first_arg .. first_arg + n_args).
 *   MS_CONST: p0 = first limb in `limbs` (u32 little-endian, ceil(width/32) limbs)
 *   MS_VAR: p0 = variable id (0..n_vars-1)
 *   MS_UF: p0 = function id; MS_ARRAY: p0 = array id; MS_K / MS_STORE / MS_ARRAY:
 *     width 0, p1 = range width (the domain is the index operand's width)
 *   MS_EXTRACT: p0 = hi, p1 = lo; MS_ZERO_EXTEND / MS_SIGN_EXTEND: p0 = bits added
 * roots: 1-bit nodes asserted true.  minimize: bit-vector nodes minimised in
 * order (lexicographic), after satisfiability.
 */
typedef struct {
    uint32_t n_nodes;
    const uint32_t *nodes;
    const uint32_t *args;
    const uint32_t *limbs;
    uint32_t n_roots;
    const uint32_t *roots;
    uint32_t n_minimize;
    const uint32_t *minimize;
    uint32_t n_vars, n_arrays, n_funcs;
} ms_query;

typedef struct {
    uint64_t max_conflicts;   /* 0: unbounded */
    uint32_t max_ms;          /* wall-clock budget, 0: unbounded */
    uint32_t minimize_ms;     /* extra budget for the objectives (best model so far on timeout) */
} ms_limits;

typedef struct {
    uint64_t vars, clauses, conflicts, decisions, propagations;
    uint32_t solves, ms;
} ms_stats;

#define MS_SAT 1
#define MS_UNSAT 0
#define MS_UNKNOWN 2          /* budget exhausted: the reference's SolverTimeOutException */
#define MS_EINVAL (-1)
#define MS_ESPACE (-2)        /* model stream larger than its buffer */

int ms_abi_version(void);

/* Decide q.  On MS_SAT the model is written to `model` (u32 words, capacity
 * `model_cap`, length in *model_len) as records
 *     {3, variable id, value limbs...}                  one per variable
 *     {1, array id, index limbs..., value limbs...}     one per array point read
 *     {2, function id, argument limbs..., value limbs...}   one per application
 *   then {0}.  Widths follow the variable / the first node of that array or
 *   function (the caller's table knows them). */
int ms_solve(const ms_query *q, const ms_limits *lim, uint32_t *model, uint32_t model_cap,
             uint32_t *model_len, ms_stats *stats);

/* Sessions: one node table and one clause database across the queries of an
 * analysis.  Each ms_session_solve appends q's nodes (q.n_nodes new ones; their
 * argument indices and roots / minimize index the whole table, node ids
 * continuing from the previous call; n_vars / n_arrays / n_funcs are session
 * totals), blasts only what is new, and decides the roots as assumptions -- the
 * clause database holds definitions and congruence lemmas only, true of every
 * query, so learnt clauses carry over.  The model stream lists every variable
 * and read blasted so far.  A session is used by one thread at a time. */
typedef struct ms_session ms_session;
int ms_session_open(ms_session **out);
void ms_session_close(ms_session *s);
int ms_session_solve(ms_session *s, const ms_query *q, const ms_limits *lim, uint32_t *model,
                     uint32_t model_cap, uint32_t *model_len, ms_stats *stats);

#ifdef __cplusplus
}
#endif
#endif
