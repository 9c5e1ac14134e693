// device_state.h — HBM layout of a lane batch and of loaded codes.
//
// Lane state is interleaved by lane so that the 64 lanes of a wave that sit at
// the same pc / stack depth touch one contiguous span per access:
//   stack    [slot][lane]      32-byte word per lane   (2 x dwordx4 per access)
//   memory   [dword][lane]     big-endian dword: EVM byte 4d+0 in bits 31..24
//   calldata [dword][lane]     same packing as memory
//   env      [word][lane]      32 bytes
//   storage  [slot][lane]      64 bytes: key limbs 0..7, value limbs 8..15
// Scalars are one array per field.  A 256-bit word is 8 little-endian u32 limbs.
#pragma once
#include <stdint.h>

struct DevLanes {
    uint32_t n;          // lanes in the batch
    uint32_t N;          // row pitch in lanes (n rounded up to 64)
    uint32_t stack_cap, mem_cap, calldata_cap, storage_cap;
    // scalars [N]
    uint32_t *code_id, *pc, *sp, *msize, *depth, *status, *aux, *steps, *flags;
    uint32_t *calldata_len, *storage_count, *ret_offset, *ret_len;
    uint32_t *sha3_count, *exp_count;
    uint64_t *gas_min, *gas_max, *gas_limit;
    // interleaved state
    uint4 *stack;        // [stack_cap][N][2]
    uint32_t *mem;       // [mem_cap/4][N]
    uint32_t *calldata;  // [calldata_cap/4][N]
    uint4 *env;          // [5][N][2]
    uint4 *storage;      // [storage_cap][N][4]
    // instruction traces (BoundedLoopsStrategy): address per popped instruction
    uint32_t trace_cap;
    uint32_t *trace_len; // [N]
    uint32_t *trace;     // [trace_cap][N]
    // function-manager records (MG_REC_*): uint32 words per lane, in execution order
    uint32_t rec_cap;
    uint32_t *rec_len;   // [N]
    uint32_t *rec;       // [rec_cap][N]
    // active_function_name (svm.py:575-637): index of the last JUMP / JUMPI landing
    // on a function entry since the upload, MG_FENT_NONE if none
    uint32_t *fent;      // [N]
};

// Symbolic planes (mg_sym_alloc): stack tags, expression arena, constants.
struct DevSym {
    uint32_t node_cap, const_cap;
    uint32_t *stag;      // [stack_cap][N]
    uint4 *node;         // [node_cap][N]
    uint4 *cval;         // [const_cap][N][2]
    uint32_t *n_nodes, *n_consts;   // [N]
    uint32_t *mtag;      // [mem_cap][N]  memory byte tags: 0, or 1 + (node << 5 | byte j)
    uint2 *sttag;        // [storage_cap][N]  storage chain entry (key, value) tags: 0 or 1 + node
};

// Taint planes (mg_taint_alloc): object handle per stack slot, annotation mask
// per object, the lane's atom count, sink and yield-class masks.
struct DevTaint {
    uint32_t obj_cap;
    const uint32_t *prog;              // [256] action word per opcode (mg_taint_program)
    const uint8_t *force;              // per code instruction (coverage layout): 1 = the host runs
                                       // this instruction's hooks (mg_taint_force), or null
    uint32_t *sobj;                    // [stack_cap][N]
    unsigned long long *omask;         // [obj_cap][N]
    uint32_t *oremap;                  // [obj_cap][N] scratch of the handle compaction
    uint32_t *n_obj, *n_fixed, *n_atoms, *tflags;   // [N] (handles below n_fixed are the host's)
    unsigned long long *sink, *ymask;          // [N]
};

// Resident initial image of a batch (mg_lanes_reset); passed to the stepping
// kernel when it re-initialises every lane itself before stepping
// (mg_run_batches), pc == nullptr otherwise.
struct DevResetImage {
    const uint32_t *pc, *depth, *status, *aux, *steps, *storage_count;
    const uint64_t *gas_min, *gas_max;
    const uint4 *storage;
};

// One loaded code (Disassembly): arrays live in one device arena.
struct DevCode {
    uint32_t n_instr;    // len(instruction_list)
    uint32_t n_bytes;    // len(bytecode) for CODESIZE / CODECOPY
    uint32_t n_jres;     // entries of the jump-resolve table (last address + 1)
    uint32_t op_off;     // u8  [n_instr]            opcode byte (0xfe = INVALID)
    uint32_t addr_off;   // u32 [n_instr]            byte address of instruction
    uint32_t push_off;   // u32 [n_instr][8]         push immediate (limbs)
    uint32_t jres_off;   // u32 [n_jres]             first index with addr >= t
    uint32_t bytes_off;  // u8  [n_bytes]            full bytecode
    uint32_t cov_off;    // u8  [n_instr]            coverage bytes
    uint32_t run_off;    // u32 [n_instr][2]         straight-line run from each instruction
    uint32_t fent_off;   // u8  [n_instr]            bit 0: index is a function entry, bit 1: index + 1 is
    uint32_t _pad;
};

// Per-launch statistics accumulated by the stepping kernel.
struct DevCounters {
    unsigned long long lane_steps;
    unsigned int running, halted, hooked, escaped;
};

#define MG_JRES_NONE 0xffffffffu
#define MG_FENT_NONE 0xffffffffu
