/*
 * mythgpu.h — C-ABI of libmythgpu.so, the MI355X batched execution core for
 * Mythril's LASER engine.
 *
 * The reference (dellalibera/mythril v0.23.18) is pure Python and has no FFI;
 * its hot path is a set of Python seams.  Each entry point
 * below names the seam it replaces; the Python host layer in mythril_amd/
 * binds them with ctypes (ctypes releases the GIL around every call).
 *
 * Conventions
 *   - every call returns 0 on success or a negative MG_E* code and never throws
 *     across the ABI; the message of the last failure is kept per context and
 *     returned by mg_last_error();
 *   - a 256-bit EVM word is 8 little-endian uint32 limbs (limb 0 = bits 0..31);
 *   - host buffers are plain lane-major arrays (mg_lane_soa); the device keeps
 *     its own lane-interleaved layout and transposes on upload/download;
 *   - one context per GPU, used from one host thread at a time.
 */
#ifndef MYTHGPU_H
#define MYTHGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MG_ABI_VERSION 15u  /* 2: model tables (arrays, uninterpreted functions)
                               3: per-lane instruction traces + loop bound
                               4: per-lane function-manager records (Keccak, EXP)
                               5: symbolic lanes: expression arena, MG_FORK
                               6: taint lanes: object handles + annotation masks
                               7: symbolic memory bytes, storage chains, symbolic
                                  SHA3 (MG_SYM_SLOAD..CONCAT, MG_REC_SYMKECCAK)
                               8: mg_lanes_download_live; kernel-2 programs keep
                                  the accumulator in operand A (bvrsub, rconcat)
                               9: mg_lanes_upload_live; lane transfers batched
                                  through one pinned DMA per phase; symbolic
                                  calldata copies (MG_SYM_CDBYTE) and a creation's
                                  calldata opcodes (MG_REC_CDSIZE) on symbolic lanes;
                                  symbolic EXP (MG_SYM_BIN 0x0a, MG_REC_SYMEXP)
                              10: MG_LANE_RETDATA (a host CALL left return data:
                                  RETURNDATASIZE / RETURNDATACOPY escape)
                              11: mg_cc_* (native conjunct compiler for kernel 2)
                              12: CALLDATACOPY of a symbolic size / memory offset /
                                  calldata offset on symbolic lanes (MG_SYM_CDBYTEX)
                              13: MLOAD / MSTORE / MSTORE8 at symbolic memory offsets
                                  (MG_SYM_MSTOREK events, MG_SYM_MLOADK reads)
                              14: SHA3 at a symbolic offset (MLOADK ranges), RETURN /
                                  REVERT of a symbolic range (MG_RET_SYMBOLIC),
                                  SELFBALANCE on MG_LANE_SYMBAL lanes, RETURNDATASIZE
                                  on MG_LANE_SYMRDS lanes, RETURNDATACOPY of a
                                  symbolic operand (pops only), BALANCE on
                                  MG_LANE_BALANCE lanes (MG_SYM_BALANCE), symbolic
                                  jump targets (JUMP: VmException, JUMPI: falls
                                  through), SHA3 of a symbolic length (MG_REC_SYMLEN),
                                  GAS / COINBASE / TIMESTAMP / DIFFICULTY on symbolic
                                  lanes (MG_ENV_GAS..MG_ENV_DIFFICULTY), NUMBER /
                                  CHAINID on MG_LANE_SYMBLOCK lanes, LOG0..4 of
                                  symbolic operands (pops only)
                              15: function-entry tracking (mg_lane_soa.fent,
                                  mg_code_fentries): the last JUMP / JUMPI landing
                                  on a dispatcher entry, for active_function_name */

/* ------------------------------------------------------------------ errors */
#define MG_OK          0
#define MG_EINVAL     -1   /* bad argument (shape, size, id)                   */
#define MG_EDEVICE    -2   /* HIP runtime failure                               */
#define MG_ENOMEM     -3   /* device or host allocation failed                  */
#define MG_ESTATE     -4   /* call out of order (e.g. step before upload)       */
#define MG_ENOCODE    -5   /* unknown code_id                                   */
#define MG_EUNSUPPORTED -6 /* a constraint the device does not evaluate (mg_cc_compile) */

/* ------------------------------------------------------------ lane status */
/* What ended (or paused) a lane.  Fields pc/sp/msize/gas of a lane that is no
 * longer RUNNING describe the state at the START of the instruction that ended
 * it — the same state the reference puts in `final_states` with track_gas=True
 * (svm.py:331-334 appends the pre-step global_state).                       */
#define MG_RUNNING        0u  /* max_steps reached, still runnable              */
#define MG_HALT_STOP      1u  /* STOP: TransactionEndSignal, world state kept   */
#define MG_HALT_RETURN    2u  /* RETURN: world state kept, ret_offset/ret_len   */
#define MG_HALT_REVERT    3u  /* REVERT: world state discarded                  */
#define MG_HALT_END       4u  /* pc past the instruction list (svm.py:384-389)  */
#define MG_HALT_DROPPED   5u  /* JUMPI true branch to invalid target: no
                                 successor and no exception (instructions.py:1614-1636) */
#define MG_VMEXC          6u  /* VmException; aux = MG_EXC_*                    */
#define MG_HOOK           7u  /* yielded before an opcode set in hook_mask      */
#define MG_ESCAPE         8u  /* needs host semantics; aux = op | reason << 8   */
#define MG_DEPTH          9u  /* strategy depth cutoff (strategy/__init__.py:29) */
#define MG_LOOP_BOUND    10u  /* BoundedLoopsStrategy dropped the state at a JUMPDEST
                                 (bounded_loops.py:119-145); aux = loop count      */

/* ret_len of a symbolic lane's RETURN / REVERT whose offset or length is symbolic
 * (instructions.py:1858-1934): the return data are the reference's fresh
 * "return_data" bytes or a slice at symbolic keys, which the host does not
 * read; LaneBatch.return_data gives None.  (A creation's RETURN of that kind
 * escapes: its return data would be the runtime code.)                     */
#define MG_RET_SYMBOLIC 0xFFFFFFFFu

#define MG_EXC_STACK_UNDERFLOW     1u
#define MG_EXC_STACK_OVERFLOW      2u
#define MG_EXC_INVALID_JUMP        3u
#define MG_EXC_INVALID_INSTRUCTION 4u
#define MG_EXC_OUT_OF_GAS          5u
#define MG_EXC_WRITE_PROTECTION    6u

#define MG_ESC_OPCODE   1u   /* opcode with symbolic or world-state semantics   */
#define MG_ESC_MEMORY   2u   /* memory would grow past the lane's page          */
#define MG_ESC_STORAGE  3u   /* storage slot table full                         */
#define MG_ESC_STACK    4u   /* stack would grow past the lane's stack_cap      */
#define MG_ESC_TRACE    5u   /* instruction trace would grow past trace_cap      */
#define MG_ESC_RECORD   6u   /* function-manager record log would grow past rec_cap */
#define MG_ESC_SYMBOLIC 7u   /* symbolic operand the device has no symbolic semantics for */
#define MG_ESC_ARENA    8u   /* the lane's expression arena / constant table is full */
#define MG_ESC_TAINT    9u   /* the lane's annotation atoms (64) or object table are full */

/* Function-manager records: what the reference registers with its global
 * function managers while a path runs, logged per lane in execution order so
 * the host can replay the registrations when it materialises the lane.
 * A record is [kind][len][step][result: 8 limbs][payload], in uint32 words;
 * step = the lane's `steps` count before the instruction (its BFS round), so
 * the host can replay registrations of all lanes in the reference's global order.
 *   MG_REC_KECCAK  SHA3 of a concrete, non-empty memory slice
 *                  (keccak_function_manager.create_keccak, keccak_function_manager.py:95-114:
 *                  concrete_hashes[data] = hash).  len = input bytes; result =
 *                  the hash; payload = ceil(len/4) words, input bytes packed
 *                  big-endian (byte 4j+0 in bits 31..24 of word j).
 *   MG_REC_EXP     EXP of concrete operands (exponent_function_manager.py:32-47:
 *                  the path gains the constraint result == Power(base, exponent),
 *                  instructions.py:624-638).  len = 0; result = base**exp mod 2^256;
 *                  payload = base limbs then exponent limbs (16 words).             */
#define MG_REC_KECCAK   1u
#define MG_REC_EXP      2u
/*   MG_REC_ANNOT   a batch-safe annotating hook the device applied (taint lanes,
 *                  mg_taint_program): len = the new atom's index; result = the
 *                  word at stack[-1] before the instruction; payload = stack[-2]
 *                  (8 limbs, 0 when absent), then pc (instruction index) and the
 *                  opcode with MG_TAINT_POST (bit 8) for a post-hook atom, then the
 *                  lane's fent (ABI v15: the hook's active_function_name).  The host
 *                  replays the module's own hook on a state built from it.        */
#define MG_REC_ANNOT    3u
/*   MG_REC_HOOK    a deferred batch-safe hook (MG_TAINT_DEFER): len = n words; result =
 *                  stack[-1]; payload = stack[-2..-n] (8 limbs each), pc, opcode, and
 *                  the lane's fent (the function name the hook sees, ABI v15).    */
#define MG_REC_HOOK     4u
/*   MG_REC_SYMKECCAK  SHA3 of a symbolic input (symbolic lanes): len = input bytes,
 *                  result limbs unused; payload = the MG_SYM_KECCAK node's index.
 *                  The host registers the input with create_keccak in the
 *                  reference's global order (symbolic_inputs).                 */
#define MG_REC_SYMKECCAK 5u
/*   MG_REC_CDSIZE  CODESIZE of a creation transaction on a symbolic lane
 *                  (instructions.py:979-1000): result = the code's size + 0x200, the
 *                  value pushed; the host appends `calldata.size == result` to the
 *                  path's constraints.  len = 0, no payload.                       */
#define MG_REC_CDSIZE   6u
/*   MG_REC_SYMEXP  EXP with a symbolic operand (symbolic lanes, instructions.py:624-638):
 *                  payload = the MG_SYM_BIN node (immediate 0x0a) pushed as the result,
 *                  Power(base, exponent); the host appends exponent_function_manager's
 *                  condition for (base, exponent) to the path.  len = 0.            */
#define MG_REC_SYMEXP   7u
/*   MG_REC_SYMLEN  SHA3 with a symbolic length (symbolic lanes, sha3_, instructions.py:
 *                  1023-1028): the length is taken as 64 and the host appends
 *                  `length == 64` to the path's constraints; len = 64, payload = the
 *                  length's arena node.  Precedes the SHA3's MG_REC_SYMKECCAK.      */
#define MG_REC_SYMLEN   8u
#define MG_REC_HEADER   11u  /* kind, len, step, 8 result limbs                */

/* lane flags */
#define MG_LANE_STATIC    1u  /* environment.static (WriteProtection)          */
#define MG_LANE_CREATION  2u  /* ContractCreationTransaction: CODE and CALLDATA ops escape */
#define MG_LANE_HOOK_ACK  4u  /* the host has fired the hooks of the instruction at pc:
                                 the first instruction of the next mg_step call runs
                                 even if its opcode is set in hook_mask; cleared by
                                 the device once that instruction has executed     */
#define MG_LANE_STEP1     8u  /* execute at most one instruction per mg_step call
                                 (the host fires post-hooks on the successor)     */
#define MG_LANE_SYMBOLIC 16u  /* symbolic lane: stepped by the symbolic stepper with
                                 stack tags and an expression arena (mg_sym_alloc) */
#define MG_LANE_SYMCD    32u  /* symbolic calldata (SymbolicCalldata): CALLDATALOAD
                                 and CALLDATASIZE make arena nodes, CALLDATACOPY escapes */
#define MG_LANE_SYMENV_SHIFT 6 /* bit 6 + MG_ENV_k: environment word k is symbolic  */
#define MG_LANE_TAINT  2048u  /* taint lane: stack words are objects with annotation
                                 sets (mg_taint_alloc); stepped by the symbolic stepper */
#define MG_LANE_SYMSTORE 4096u /* symbolic lane whose storage base is the symbolic
                                 Array("Storage{address}") (account.py:26-29), not K(0) */
#define MG_LANE_MEMTAG 8192u  /* symbolic lane whose memory may hold symbolic bytes
                                 (mtag); set by the host or by the device on a write */
#define MG_LANE_RETDATA 16384u /* the path's last_return_data is set (a CALL the host's
                                 escape handler ran): RETURNDATASIZE and RETURNDATACOPY
                                 escape; without it they push 0 / pop only, as the
                                 reference does with last_return_data None
                                 (instructions.py:1314-1370)                       */

/* environment words, per lane */
#define MG_LANE_SYMBAL 32768u /* symbolic lane whose active account's balance is
                                 symbolic: SELFBALANCE pushes an MG_SYM_ENV node
                                 (w = MG_ENV_SELFBALANCE, instructions.py:968-976) */
#define MG_LANE_SYMRDS 65536u /* symbolic lane whose last_return_data has a symbolic
                                 size (a host CALL's returndatasize variable):
                                 RETURNDATASIZE pushes an MG_SYM_ENV node
                                 (w = MG_ENV_RETURNDATASIZE, instructions.py:1359-1370) */
#define MG_LANE_SYMBLOCK 262144u /* symbolic lane whose environment's block_number and chainid are
                                    symbolic: NUMBER / CHAINID push MG_SYM_ENV nodes          */
#define MG_LANE_BALANCE 131072u /* symbolic lane of a LaserEVM with no dynamic loader: BALANCE
                                   pushes an MG_SYM_BALANCE node (the world state's accounts
                                   cannot change inside a device run)                    */
#define MG_ENV_ADDRESS   0
#define MG_ENV_CALLER    1
#define MG_ENV_ORIGIN    2
#define MG_ENV_CALLVALUE 3
#define MG_ENV_GASPRICE  4
#define MG_ENV_WORDS     5
#define MG_ENV_SELFBALANCE 5  /* MG_SYM_ENV immediate only: environment.active_account.balance() */
#define MG_ENV_RETURNDATASIZE 6 /* MG_SYM_ENV immediate only: last_return_data.size */
#define MG_ENV_GAS 7           /* MG_SYM_ENV immediate only: new_bitvec("gas", 256) (gas_, instructions.py:1700-1709) */
#define MG_ENV_COINBASE 8      /* ... new_bitvec("coinbase", 256) (coinbase_, :1386-1393)                      */
#define MG_ENV_TIMESTAMP 9     /* ... new_bitvec("timestamp", 256) (timestamp_, :1396-1403)                    */
#define MG_ENV_DIFFICULTY 10   /* ... new_bitvec("block_difficulty", 256) (difficulty_, :1416-1425)            */
#define MG_ENV_NUMBER 11       /* ... environment.block_number (number_, :1406-1413), on MG_LANE_SYMBLOCK lanes  */
#define MG_ENV_CHAINID 12      /* ... environment.chainid (chainid_, :958-965), on MG_LANE_SYMBLOCK lanes        */

#define MG_STACK_LIMIT 1024u              /* MachineStack.STACK_LIMIT           */
#define MG_MSTATE_GAS_LIMIT 1000000000ull /* GlobalState default gas_limit      */

/* ------------------------------------------------------- host lane layout */
/* Lane-major host image of a batch of concrete EVM paths.  Any pointer may be
 * NULL on download to skip that field.                                     */
typedef struct mg_lane_soa {
    uint32_t n;             /* lanes described by the arrays below            */
    uint32_t stack_cap;     /* stack entries per lane in `stack`              */
    uint32_t mem_cap;       /* bytes per lane in `memory` (multiple of 32)    */
    uint32_t calldata_cap;  /* bytes per lane in `calldata`                   */
    uint32_t storage_cap;   /* slots per lane in `storage`                    */
    uint32_t _pad;
    uint32_t *code_id;      /* [n]                                             */
    uint32_t *pc;           /* [n] instruction INDEX (Appendix A #1)          */
    uint32_t *sp;           /* [n] stack depth                                */
    uint32_t *msize;        /* [n] memory size in bytes                       */
    uint32_t *depth;        /* [n] JUMPI depth (mstate.depth)                 */
    uint32_t *status;       /* [n] MG_RUNNING / MG_HALT_* / ...               */
    uint32_t *aux;          /* [n] exception kind / escape op|reason / hook op */
    uint32_t *steps;        /* [n] lane-steps executed (cumulative)           */
    uint32_t *flags;        /* [n] MG_LANE_*                                  */
    uint64_t *gas_min;      /* [n] mstate.min_gas_used                        */
    uint64_t *gas_max;      /* [n] mstate.max_gas_used                        */
    uint64_t *gas_limit;    /* [n] transaction gas_limit                      */
    uint32_t *calldata_len; /* [n]                                             */
    uint8_t  *calldata;     /* [n][calldata_cap]                              */
    uint32_t *env;          /* [n][MG_ENV_WORDS][8]                           */
    uint32_t *stack;        /* [n][stack_cap][8]   slot 0 = bottom            */
    uint8_t  *memory;       /* [n][mem_cap]                                    */
    uint32_t *storage_count;/* [n]                                             */
    uint32_t *storage;      /* [n][storage_cap][16] key limbs 0..7, value 8..15 */
    uint32_t *ret_offset;   /* [n] RETURN/REVERT data offset (low 32 bits)    */
    uint32_t *ret_len;      /* [n] RETURN/REVERT data length (low 32 bits)    */
    /* JumpdestCountAnnotation.trace (bounded_loops.py:14-26): the byte address of
     * every instruction the path has been popped at, when traces are on       */
    uint32_t trace_cap;     /* entries per lane in `trace` (0: no traces)      */
    uint32_t _pad2;
    uint32_t *trace_len;    /* [n]                                             */
    uint32_t *trace;        /* [n][trace_cap]                                  */
    /* function-manager records (MG_REC_*), in execution order                  */
    uint32_t rec_cap;       /* uint32 words per lane in `rec` (0: not recorded) */
    uint32_t _pad3;
    uint32_t *rec_len;      /* [n] words used                                  */
    uint32_t *rec;          /* [n][rec_cap]                                    */
    /* LaserEVM._new_node_state (svm.py:575-637): after every JUMP / JUMPI the
     * successor's instruction address switches environment.active_function_name
     * when it is a dispatcher entry (Disassembly.address_to_function_name,
     * disassembly.py:36-56) or address 0 ("fallback").  The device keeps the
     * instruction INDEX of the last such landing since the upload, or
     * MG_FENT_NONE; the host maps it to the name.  NULL: uploads MG_FENT_NONE,
     * downloads nothing (ABI <= 14 callers).                                  */
    uint32_t *fent;         /* [n]                                             */
} mg_lane_soa;
#define MG_FENT_NONE 0xffffffffu

/* Per-call statistics of mg_step. */
typedef struct mg_step_stats {
    uint64_t lane_steps;    /* instructions executed by all lanes in the call */
    uint32_t running;       /* lanes still MG_RUNNING after the call          */
    uint32_t halted;        /* lanes in a terminal status                     */
    uint32_t hooked;        /* lanes in MG_HOOK                               */
    uint32_t escaped;       /* lanes in MG_ESCAPE                             */
    float    kernel_ms;     /* device time of the stepping kernel(s)          */
    uint32_t launches;      /* kernel launches issued                         */
} mg_step_stats;

/* Batch configuration, fixed at mg_lanes_alloc. */
typedef struct mg_batch_cfg {
    uint32_t n_lanes;
    uint32_t stack_cap;     /* <= MG_STACK_LIMIT                              */
    uint32_t mem_cap;       /* bytes, multiple of 32                           */
    uint32_t calldata_cap;  /* bytes                                           */
    uint32_t storage_cap;   /* slots                                           */
    uint32_t coverage;      /* 1: record the per-code coverage bitmap         */
    uint32_t trace_cap;     /* instruction-trace entries per lane (0: none)   */
    uint32_t rec_cap;       /* function-manager record words per lane (0: none) */
} mg_batch_cfg;

typedef struct mg_ctx mg_ctx;

/* ---------------------------------------------------------- symbolic lanes
 * A symbolic lane keeps every stack word's value plus a tag: 0 = concrete,
 * else 1 + the index of the arena node that defines it.  Arena node = 4 u32:
 *   x = kind | width << 8 (width 1: a Bool, 256: a bit-vector),
 *   y, z = operand refs (MG_SYM_CONST | k: entry k of the lane's constant
 *          table; else a node index), w = immediate (EVM opcode / env word).
 * Kinds (the host builds the reference's expression for each, see
 * mythril_amd/laser/symbolic.py): */
#define MG_SYM_CDLOAD 1u  /* calldata.get_word_at(y) (state/calldata.py:214-262)  */
#define MG_SYM_CDSIZE 2u  /* calldata.calldatasize                               */
#define MG_SYM_ENV    3u  /* environment word w (MG_ENV_*)                       */
#define MG_SYM_BIN    4u  /* binary EVM opcode w on (y = first pop, z = second)  */
#define MG_SYM_UN     5u  /* unary EVM opcode w (ISZERO, NOT) on y               */
#define MG_SYM_SLOAD  6u  /* simplify(Select(store chain after its first z entries, y))
                             (account.py:43-75, instructions.py:1496-1506)        */
#define MG_SYM_KECCAK 7u  /* keccak256_w(y): create_keccak of a symbolic input of w bits
                             (keccak_function_manager.py:95-114, instructions.py:1013-1051) */
#define MG_SYM_EXTRACT 8u /* Extract(w >> 16, w & 0xffff, y) of a node's word      */
#define MG_SYM_CONCAT 9u  /* Concat(y, z), widths w & 0xffff and w >> 16: the parts of
                             a memory read, simplify(Concat(bytes)) (memory.py:56-82) */
#define MG_SYM_TERM  10u  /* an opaque term of the host's expression layer, index w in
                             the host's term table (anything a handler or the caller
                             built); compared by identity                          */
#define MG_SYM_CDBYTE 12u /* calldata[w]: one 8-bit byte of the calldata, If(w < size,
                             calldata_array[w], 0) (state/calldata.py:253-262), as
                             _calldata_copy_helper writes it (instructions.py:807-875) */
#define MG_SYM_CDBYTEX 13u /* calldata[simplify(y + w)]: byte w of a CALLDATACOPY from a
                              symbolic calldata offset y (instructions.py:816-860; a
                              symbolic size copies 320 bytes, call.py:33)           */
#define MG_SYM_MSTOREK 14u /* an event, not a term: a write at the symbolic memory offset y
                              of value ref z -- w = 1: MSTORE (write_word_at), 2: MSTORE8
                              (the value's low byte), 3: one byte (a host-encoded key).  The
                              lane's events in arena order are its byte map at symbolic keys
                              (memory.py:117-203, keys simplify(index))                    */
#define MG_SYM_MLOADK 15u  /* a read at the symbolic offset y over the byte map the events
                              before this node build: w = 0, memory.get_word_at(y) (MLOAD,
                              instructions.py:1439-1451); w = n > 0, simplify(Concat(memory[y :
                              y + n])) (the data of a SHA3, instructions.py:1014-1051)     */
#define MG_SYM_BALANCE 16u /* BALANCE of the address ref y (balance_, instructions.py:907-931,
                              no dynamic loader): the account's balance() when y is a known
                              concrete address, else the If chain over the world state's
                              accounts; on MG_LANE_BALANCE lanes                           */
#define MG_SYM_CONST  0x80000000u
#define MG_FORK      11u  /* status: JUMPI on a symbolic condition; the lane holds
                             the state at the start of the JUMPI (host forks)    */

/* Host image of the symbolic planes of lanes [first, first + n), lane-major.
 * Memory bytes and storage entries carry tags too (ABI v7): a memory byte tag is
 * 0 (the byte in `memory` is the value) or 1 + (node << 5 | j): byte j (0 = most
 * significant) of that node's word, i.e. Extract(255 - 8j, 248 - 8j, word) as
 * write_word_at stores it (memory.py:84-115).  In a symbolic lane the storage
 * table is the reference's store chain, one entry per SSTORE in order (over K(0),
 * or the symbolic Array with MG_LANE_SYMSTORE); an entry's key / value tag is 0
 * (the limbs are the value) or 1 + node. */
typedef struct mg_sym_soa {
    uint32_t n, stack_cap, node_cap, const_cap;
    uint32_t *stag;         /* [n][stack_cap]                                 */
    uint32_t *node;         /* [n][node_cap][4]                               */
    uint32_t *cval;         /* [n][const_cap][8] little-endian limbs          */
    uint32_t *n_nodes;      /* [n]                                            */
    uint32_t *n_consts;     /* [n]                                            */
    uint32_t mem_cap, storage_cap;   /* the lane image's capacities               */
    uint32_t *mtag;         /* [n][mem_cap] memory byte tags                  */
    uint32_t *sttag;        /* [n][storage_cap][2] storage entry (key, value) tags */
} mg_sym_soa;

/* Symbolic planes for the current batch (after mg_lanes_alloc; freed with it).
 * Lanes flagged MG_LANE_SYMBOLIC are stepped by the symbolic stepper in the same
 * mg_step / mg_step_until call, right after the concrete stepper. */
int         mg_sym_alloc(mg_ctx *ctx, uint32_t node_cap, uint32_t const_cap);
int         mg_sym_upload(mg_ctx *ctx, const mg_sym_soa *host, uint32_t first, uint32_t n);
int         mg_sym_download(mg_ctx *ctx, mg_sym_soa *host, uint32_t first, uint32_t n);

/* ------------------------------------------------------------ taint lanes
 * The reference's stack words are Python objects carrying a mutable set of
 * annotations (laser/smt/expression.py:10-57): ALU results take the union of
 * their operands' sets (bitvec.py:63-136), DUP pushes the SAME object
 * (instructions.py:330) so a later annotate() on it shows on every copy, the
 * environment words are one object each (instructions.py:895-1060), and concrete
 * memory / storage round trips drop them (memory.py:84-115, account.py:43-87).
 * A taint lane (MG_LANE_TAINT) reproduces that on the device: every stack slot
 * holds an object handle (0: an object no other slot shares and that has no
 * annotations; 1..5: the environment words MG_ENV_k + 1; 6: the symbolic
 * calldata size; >= 7: the lane's object table), and every object an annotation
 * mask over the lane's atoms (<= 64; the host maps atom k to annotation objects).
 *
 * Batch-safe hooks (mythril_amd/laser/taint.py) become per-opcode actions the
 * device applies instead of yielding to the host, and log an MG_REC_ANNOT record
 * per new atom.  Action word per opcode byte (mg_taint_program): */
#define MG_TAINT_PRE_SHIFT   0   /* bits 0..3: operand k + 1 of a pre-hook that annotates stack[-1-k] */
#define MG_TAINT_POST       16u  /* a post-hook annotates the pushed word                     */
#define MG_TAINT_EXPCOND    32u  /* skip the pre-annotation when stack[-2] == 0 or stack[-1] < 2
                                    (integer.py:161-166)                                        */
#define MG_TAINT_YCLASS     64u  /* this action's atoms join the lane's yield class            */
#define MG_TAINT_SINK_SHIFT  8   /* bits 8..11: operand k + 1 whose set a pre-hook adds to the
                                    state annotation (the lane's sink mask)                    */
#define MG_TAINT_YIELD_SHIFT 12  /* bits 12..15: operand k + 1: yield (MG_HOOK) only when that
                                    word carries an atom of the yield class                   */
#define MG_TAINT_DEFER_SHIFT 16  /* bits 16..19: 1..3: a pre-hook replayed later from a record of
                                    stack[-1..-n] (MG_REC_HOOK); it reads only those words     */
#define MG_TAINT_IFSYM_SHIFT 20  /* bits 20..23: operand k + 1: a pre-hook with work only when that
                                    word is symbolic (yield then)                              */
#define MG_TAINT_IFLANE     (1u << 24)  /* yield when the lane's tflags bit 1 is set (a state
                                    annotation the host found at pack)                          */
#define MG_TAINT_OBJ0        7u  /* first object-table handle                                  */

/* Host image of the taint planes of lanes [first, first + n), lane-major. */
typedef struct mg_taint_soa {
    uint32_t n, stack_cap, obj_cap, _pad;
    uint32_t *sobj;         /* [n][stack_cap] object handle per stack slot      */
    uint64_t *omask;        /* [n][obj_cap]   annotation mask per object         */
    uint32_t *n_obj;        /* [n] object handles in use (>= MG_TAINT_OBJ0)     */
    uint32_t *n_fixed;      /* [n] handles below this are the host's objects: the
                               device's handle compaction never renumbers them  */
    uint32_t *n_atoms;      /* [n] atoms in use (<= 64)                          */
    uint64_t *sink;         /* [n] atoms the sink hooks collected                */
    uint64_t *ymask;        /* [n] atoms of the yield class                      */
    uint32_t *tflags;       /* [n] bit 0: a sink hook ran; bit 1: MG_TAINT_IFLANE yields */
} mg_taint_soa;

/* Taint planes for the current batch (after mg_lanes_alloc; freed with it) and
 * the per-opcode action table (256 words; zeros = no batch-safe hooks). */
int         mg_taint_alloc(mg_ctx *ctx, uint32_t obj_cap);
int         mg_taint_program(mg_ctx *ctx, const uint32_t actions[256]);
/* Per instruction of a code (n = its instruction count): 1 = a taint lane stops
 * there with MG_HOOK instead of applying the opcode's actions, 2 = it applies
 * none (addresses in modules' issue caches, where DetectionModule.execute returns
 * early, base.py:79-86: 2 when every module on the opcode has it cached). */
int         mg_taint_force(mg_ctx *ctx, uint32_t code_id, const uint8_t *flags, uint32_t n);
int         mg_taint_upload(mg_ctx *ctx, const mg_taint_soa *host, uint32_t first, uint32_t n);
int         mg_taint_download(mg_ctx *ctx, mg_taint_soa *host, uint32_t first, uint32_t n);

/* ------------------------------------------------------------- lifecycle */
int         mg_abi_version(void);
int         mg_open(int device, mg_ctx **out);
void        mg_close(mg_ctx *ctx);
const char *mg_last_error(mg_ctx *ctx);
/* Opcode table the device uses (support/opcodes.py:16-144 + instruction_data.py:
 * 51-56): gas (min,max) and required stack items for a byte, or -1 if the
 * byte disassembles to INVALID (asm.py:126-131).                            */
int         mg_opcode_info(uint32_t byte, uint32_t *gas_min, uint32_t *gas_max,
                           uint32_t *stack_req);

/* ------------------------------------------------------------------ code */
/* Replaces Disassembly(code) (disassembly.py:9-56, asm.py:99-148) +
 * util.get_instruction_index (util.py:45-59): builds the instruction table
 * (pc = index), push immediates, the ">="-jump-resolve table and keeps the
 * full bytecode for CODECOPY/CODESIZE.                                        */
int         mg_load_code(mg_ctx *ctx, const uint8_t *code, size_t n, uint32_t *code_id);
/* Number of instructions of a loaded code (len(instruction_list)).          */
int         mg_code_info(mg_ctx *ctx, uint32_t code_id, uint32_t *n_instr);
/* The device's function-entry flags of a loaded code, one byte per instruction
 * (n = its instruction count): bit 0 = a JUMP / JUMPI landing on this index
 * switches active_function_name (an entry of the PUSH1..4 EQ PUSHn dispatcher
 * pattern, asm.py:66-94 + disassembly.py:36-56 / 64-114, or index 0 =
 * address 0), bit 1 = the same for the next index (JUMPI fall-through).      */
int         mg_code_fentries(mg_ctx *ctx, uint32_t code_id, uint8_t *out, uint32_t n);
/* The device's instruction table of a loaded code (n = its instruction count):
 * opcode byte per index (0xfe for bytes asm.py:126-131 disassembles to INVALID)
 * and the byte address of each instruction -- Disassembly.instruction_list
 * without the arguments (they are the code's bytes after each PUSH).          */
int         mg_code_table(mg_ctx *ctx, uint32_t code_id, uint8_t *ops, uint32_t *addrs, uint32_t n);

/* ----------------------------------------------------------------- lanes */
int         mg_lanes_alloc(mg_ctx *ctx, const mg_batch_cfg *cfg);
/* Upload lanes [first, first+n) from host (host->n must equal n).  The
 * upload also becomes the batch's resident initial image (see mg_lanes_reset). */
int         mg_lanes_upload(mg_ctx *ctx, const mg_lane_soa *host, uint32_t first, uint32_t n);
int         mg_lanes_download(mg_ctx *ctx, mg_lane_soa *host, uint32_t first, uint32_t n);
/* mg_lanes_download of what the lanes can have changed, for a host image that
 * was uploaded from the same buffers: the scalars, then each lane's stack rows
 * below the largest sp of the range, memory below the largest msize, storage
 * entries below the largest storage_count, records below the largest rec_len
 * and trace entries below the largest trace_len.  calldata and the environment
 * words (never written by a step) and everything above those bounds keep the
 * host's contents.  The batched LaserEVM's per-launch copy-back
 * (svm.py:293-337 drain) -- a full download moves every lane's whole stack.  */
int         mg_lanes_download_live(mg_ctx *ctx, mg_lane_soa *host, uint32_t first, uint32_t n);
/* mg_lanes_upload of what a step reads: the scalars, calldata and environment
 * words whole, each lane's stack rows below the largest sp of the range,
 * memory below the largest msize (a step zero-fills memory it extends),
 * storage entries below the largest storage_count, trace entries below the
 * largest trace_len and records below the largest rec_len; device rows above
 * those bounds keep their contents.  The batched LaserEVM's per-launch upload
 * of the lanes its host hooks touched (svm.py:369-491 resume).               */
int         mg_lanes_upload_live(mg_ctx *ctx, const mg_lane_soa *host, uint32_t first, uint32_t n);
/* Re-initialise every lane from the resident initial image on the device
 * (no host traffic): pc, sp, msize, gas, status, storage, steps.            */
int         mg_lanes_reset(mg_ctx *ctx);

/* Replaces the LaserEVM.exec() drain for device-eligible lanes (svm.py:293-337
 * + execute_state svm.py:369-491 + Instruction.evaluate instructions.py:235-267):
 * steps every RUNNING lane until it halts, escapes, reaches an opcode whose bit
 * is set in hook_mask (bit b of hook_mask[b>>6]), or has executed max_steps
 * instructions in this call.  max_depth: states with depth >= max_depth are
 * dropped (0 = unlimited).                                                   */
int         mg_step(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps,
                    uint32_t max_depth, mg_step_stats *stats);
/* BoundedLoopsStrategy (bounded_loops.py:84-145) on the device: with bound > 0
 * (and a batch allocated with trace_cap > 0) every instruction a lane is popped
 * at is appended to its trace, and at a JUMPDEST a lane whose loop count
 * (get_loop_count) exceeds the bound stops with MG_LOOP_BOUND; creation lanes
 * only when the count also reaches 128.  0 turns it off.                      */
int         mg_set_loop_bound(mg_ctx *ctx, uint32_t bound);
/* Same, with a step horizon: a lane also pauses (stays MG_RUNNING) once its
 * cumulative `steps` reaches `horizon` (0 = none).  The host layer uses it to
 * deliver hook and halt events in the reference's BFS round order
 * (mythril_amd/laser/svm.py).                                                */
int         mg_step_until(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps,
                          uint32_t max_depth, uint32_t horizon, mg_step_stats *stats);
/* n_batches whole batches enqueued back to back with one host wait: for each,
 * mg_lanes_reset then one stepping launch, statistics into stats[b] (kernel_ms
 * = the sequence's device time / n_batches, launch gaps included; with
 * MG_BATCH_EVENTS=1 each launch is bracketed instead).  Same preconditions as
 * mg_lanes_reset.                                                           */
int         mg_run_batches(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps,
                           uint32_t max_depth, uint32_t n_batches, mg_step_stats *stats);
/* Profiling variant (the InstructionProfiler plugin's per-opcode counts,
 * instruction_profiler.py:41-115, as native counters): op_counts[256] =
 * instructions executed per opcode byte; extra[4] = {SHA3 input bytes,
 * CALLDATACOPY/CODECOPY bytes, storage entries scanned, Keccak blocks}.     */
int         mg_step_profile(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps,
                            uint32_t max_depth, uint64_t *op_counts, uint64_t *extra);
/* Same, asynchronous: enqueue only (no stats, no host sync).                */
int         mg_step_async(mg_ctx *ctx, const uint64_t hook_mask[4], uint32_t max_steps,
                          uint32_t max_depth);
int         mg_sync(mg_ctx *ctx);

/* Coverage plugin state (coverage_plugin.py:68-85): one byte per instruction
 * index, 1 = executed by some lane since the last mg_coverage_clear.         */
int         mg_coverage(mg_ctx *ctx, uint32_t code_id, uint8_t *bytes, uint32_t n);
int         mg_coverage_clear(mg_ctx *ctx);

/* Number of Keccak-256 evaluations (SHA3 with concrete input) and EXP
 * evaluations per lane since upload/reset: the host re-registers them with
 * keccak_function_manager / exponent_function_manager when it materialises a
 * lane as a GlobalState (keccak_function_manager.py:95-114).                 */
int         mg_event_counts(mg_ctx *ctx, uint32_t *sha3_count, uint32_t *exp_count,
                            uint32_t first, uint32_t n);

/* -------------------------------------------------- constraint prefilter */
/* A batch of constraint sets, each compiled by the host into a register
 * program over 256-bit values (mythril_amd/smt/flatten.py).  Replaces the
 * model loop of ModelCache.check_quick_sat (support_utils.py:60-68).
 * Instruction: op | width << 8 | store << 17 | slot << 18, then three operand
 * refs (kind << 30 | index; kind 0 = the accumulator, 1 slot, 2 variable,
 * 3 constant) or immediates.  Since ABI 8 only operand A may be the
 * accumulator (the flattener swaps / reverses / spills): a program with the
 * accumulator in operand B or C is refused with MG_EINVAL, and so is one
 * with any of bits 22..31 of the first word set (the library's own fused
 * forms use them: it rewrites common instruction pairs and chains into
 * superinstructions at upload, bit-identical results; MG_BV_FUSE=0 disables). */
typedef struct mg_dag_batch {
    uint32_t n_dags;
    uint32_t n_slots;       /* register slots a program may use (<= 16)       */
    const uint32_t *prog_off;   /* [n_dags+1] offsets into `insns`            */
    const uint32_t *insns;      /* [total][4] encoded instructions            */
    const uint32_t *consts;     /* [n_consts][8] 256-bit constants            */
    uint32_t n_consts;
} mg_dag_batch;

/* Candidate models, most-recently-used first (LRU order of
 * support_utils.py:62-63).  Variables absent from a model take 0
 * (z3 model_completion).  The values table (n_vars x
 * n_models x 32 bytes) must stay under 4 GiB: the kernel addresses it with
 * 32-bit offsets, and a larger one is refused with MG_EINVAL.
 *
 * Tables are the models' interpretations of symbolic arrays (storage,
 * calldata, balances: array.py) and uninterpreted functions (keccak256_N and
 * its inverse, Power: function.py), looked up by the program op BV_TAB.  For
 * table t and model m, entries [tab_start[t][m], + tab_count[t][m]) of
 * tab_entries hold (key k0: 8 limbs, key k1: 8 limbs, value: 16 limbs, i.e. up
 * to 512 bits); a key not listed takes tab_default[t][m] (array default /
 * function else value).                                                     */
typedef struct mg_model_batch {
    uint32_t n_models;
    uint32_t n_vars;
    const uint32_t *values;     /* [n_vars][n_models][8]                      */
    uint32_t n_tables;          /* 0: no tables (pointers below ignored)      */
    const uint32_t *tab_start;  /* [n_tables][n_models]                       */
    const uint32_t *tab_count;  /* [n_tables][n_models]                       */
    const uint32_t *tab_entries;/* [n_entries][32]                            */
    uint32_t n_entries;
    const uint32_t *tab_default;/* [n_tables][n_models][16]                   */
} mg_model_batch;

/* first_sat_model[d] = smallest model index m (MRU order) whose evaluation of
 * DAG d is true, UINT32_MAX if none; sat_count[d] = number of satisfying
 * models (may be NULL).                                                      */
int         mg_eval(mg_ctx *ctx, const mg_dag_batch *dags, const mg_model_batch *models,
                    uint32_t *first_sat_model, uint32_t *sat_count, float *kernel_ms);

/* Same, plus the full satisfaction bitmap: bit m of sat_bits[d][m / 64] is set
 * when model m satisfies DAG d (sat_bits: [n_dags][ceil(n_models / 64)]).  With
 * it the host replays a sequence of check_quick_sat calls exactly, including
 * the LRU moves of returned models between calls (support_utils.py:60-68).    */
int         mg_eval_bits(mg_ctx *ctx, const mg_dag_batch *dags, const mg_model_batch *models,
                         uint32_t *first_sat, uint32_t *sat_count, uint64_t *sat_bits,
                         float *kernel_ms);

/* Device-resident variant used by the benchmark: upload once, evaluate many
 * times without host traffic. */
int         mg_eval_upload(mg_ctx *ctx, const mg_dag_batch *dags, const mg_model_batch *models);
int         mg_eval_run(mg_ctx *ctx, uint32_t dag_first, uint32_t dag_count, float *kernel_ms);
int         mg_eval_download(mg_ctx *ctx, uint32_t *first_sat_model, uint32_t *sat_count,
                             uint32_t dag_first, uint32_t dag_count);

/* ------------------------------------------------------ conjunct compiler */
/* Kernel 2's register programs compiled on the host from lowered constraint
 * DAGs (mythril_amd/smt/flatten.py's passes in native code; replaces the
 * Python compile of every quick-sat query's conjuncts, support/model.py:48-56
 * -> get_model's And(constraints)).  Nodes are registered once each into a
 * growing table (ids only grow), programs are compiled per conjunct root.
 * Host only: no device, no context needed.                                  */
typedef struct mg_cc mg_cc;
int         mg_cc_open(mg_cc **out);
void        mg_cc_close(mg_cc *cc);
const char *mg_cc_error(mg_cc *cc);
/* rows: n x {op, width, first_arg, n_args, imm}; op = a kernel-2 opcode
 * (bv_eval.cuh BV_*), or 0x1000 (variable: imm = its model-pool index) /
 * 0x1001 (constant: imm = its constant-pool index).  args[first_arg ..]: node
 * ids, or 0x80000000 | k for row k of this call.  ids[i] <- row i's id (an
 * equal existing node's id when there is one).  imm: the low bit of an
 * extract; table index | part << 20 | low bit << 21 of a table lookup.      */
int         mg_cc_add(mg_cc *cc, const uint32_t *rows, uint32_t n, const uint32_t *args, uint32_t n_args,
                      uint32_t *ids);
/* The program of the conjunct rooted at node `root`: n_insns x 4 u32 into
 * insns (cap instructions); *max_slots is raised to the slots it uses.
 * MG_EUNSUPPORTED: more than 16 live values, more than 2048 instructions or
 * a value wider than 256 bits (the set stays with the SMT backend).        */
int         mg_cc_compile(mg_cc *cc, uint32_t root, uint32_t *insns, uint32_t cap, uint32_t *n_insns,
                          uint32_t *max_slots);

#ifdef __cplusplus
}
#endif
#endif /* MYTHGPU_H */
