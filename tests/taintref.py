"""Object-level restatement of the reference's annotation semantics on taint lanes
-- TEST INFRASTRUCTURE ONLY (the checker for kernel 1's taint planes, and the
stand-in for k_sym_step's taint lanes in tests/oracle_device.py).

The reference keeps stack words as Python objects with annotation sets.  This
file restates what each executed instruction does to those objects, from the
reference's handlers:

* DUPn pushes ``stack[-n]`` itself (instructions.py:325-331); SWAPn swaps the two
  references (:333-338); POP drops one (:340-343);
* ADDRESS / CALLER / ORIGIN / CALLVALUE / GASPRICE push the environment's own
  object (:895-905, 934-955, 1054-1061);
* the ALU handlers build a new object whose set is the union of the popped
  operands' (bitvec.py:63-136, bitvec_helper.py If/Concat/Extract/URem...):
  ADD SUB MUL EXP SIGNEXTEND LT GT SLT SGT EQ AND OR XOR SHL SHR SAR over two,
  ADDMOD MULMOD over three, ISZERO NOT over one; DIV SDIV MOD SMOD push a fresh 0
  when the divisor is 0 (:505-592); BYTE keeps only the value's set, and pushes a
  fresh 0 for an index past the word (:426-456);
* every other push is a fresh object (concrete memory, storage, calldata,
  Keccak, constants: memory.py:84-115, account.py:43-87, array.py:21-28);

plus the batch-safe hook actions of mythril_amd/laser/taint.py restated at the
object level: a pre-hook annotate() adds a new atom to ``stack[-1-k]`` itself
(integer.py:140-186, with EXP's early return), a sink hook collects
``stack[-1-k]``'s set (integer.py:204-226), a post-hook annotates the pushed
object, a yield-if hook stops the lane when its operand carries a yield-class
atom.  Values, gas, halts and every other effect come from the C oracle
(oracle/evm_ref.c), stepped one instruction at a time.

Objects are Python objects here (identity = ``is``), atoms small ints; the
device's handle numbers are its own business, so the GPU test compares the
*partition* of stack slots into objects and each slot's atom set.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from mythril_amd.lanes import (MG_ESC_OPCODE, MG_ESC_RECORD, MG_ESC_TAINT, MG_ESCAPE, MG_HOOK,
                               MG_LANE_HOOK_ACK, MG_LANE_STEP1, MG_REC_ANNOT, MG_REC_ANNOT_WORDS, MG_REC_HOOK,
                               MG_TAINT_IFLANE,
                               MG_REC_HEADER, MG_RUNNING, MG_TAINT_CDSIZE, MG_TAINT_EXPCOND,
                               MG_TAINT_OBJ0, MG_TAINT_POST, MG_TAINT_YCLASS, limbs_to_word,
                               word_to_limbs)

ENV_OPS = {0x30: 1, 0x33: 2, 0x32: 3, 0x34: 4, 0x3A: 5}
UNION2 = {0x01, 0x02, 0x03, 0x0A, 0x0B, 0x10, 0x11, 0x12, 0x13, 0x14, 0x16, 0x17, 0x18, 0x1B, 0x1C, 0x1D}
ZERODIV = {0x04, 0x05, 0x06, 0x07}
# opcodes whose mutator pushes nothing (instructions.py)
NO_PUSH = {0x00, 0x37, 0x39, 0x3E, 0x50, 0x52, 0x53, 0x55, 0x56, 0x57, 0x5B, 0xA0, 0xA1, 0xA2, 0xA3, 0xA4,
           0xF3, 0xFD, 0xFE, 0xFF}


class Obj:
    """A stack word.  `tracked`: the device has given it an object handle (it was
    DUP'd, annotated, or made with annotations) -- only the object-table
    capacity check (MG_ESC_TAINT) depends on it."""
    __slots__ = ("ann", "tracked")

    def __init__(self, ann=(), tracked=None):
        self.ann = set(ann)
        self.tracked = bool(self.ann) if tracked is None else tracked


def _bits(m: int):
    return {k for k in range(64) if (int(m) >> k) & 1}


def _mask(s) -> int:
    m = 0
    for k in s:
        m |= 1 << k
    return m


class RefLane:
    """One lane's objects, read from (and written back to) a LaneBatch's planes."""

    def __init__(self, b, i: int):
        self.fixed: Dict[int, Obj] = {}
        self.env: Dict[int, Obj] = {}
        for h in range(1, MG_TAINT_CDSIZE + 1):
            self.env[h] = Obj(_bits(b.omask[i, h]))
        self.stack: List[Obj] = []
        for s in range(int(b.sp[i])):
            h = int(b.sobj[i, s])
            if h == 0:
                self.stack.append(Obj())
            elif h < MG_TAINT_OBJ0:
                self.stack.append(self.env[h])
            else:
                if h not in self.fixed:
                    self.fixed[h] = Obj(_bits(b.omask[i, h]), tracked=True)
                self.stack.append(self.fixed[h])
        self.n_fixed = int(b.n_fixed[i])
        self.n_obj = int(b.n_obj[i])
        self.natoms = int(b.n_atoms[i])
        self.sink = _bits(b.sink[i])
        self.tflags = int(b.tflags[i])
        self.ymask = _bits(b.ymask[i])

    def write(self, b, i: int) -> None:
        """Planes for these objects: existing handles stay, new objects get handles
        from n_obj on in order of first appearance (the device allocates past
        every handle in use)."""
        b.omask[i] = 0
        for h, o in self.env.items():
            b.omask[i, h] = _mask(o.ann)
        handle = {id(o): h for h, o in self.env.items()}
        for h, o in self.fixed.items():
            handle[id(o)] = h
            b.omask[i, h] = _mask(o.ann)
        nxt = self.n_obj
        b.sobj[i] = 0
        count: Dict[int, int] = {}
        for o in self.stack:
            count[id(o)] = count.get(id(o), 0) + 1
        new = sum(1 for o in {id(x): x for x in self.stack}.values()
                  if id(o) not in handle and (count[id(o)] > 1 or o.ann))
        if nxt + new + 4 > b.shape.obj_cap:
            # the device's compaction: handles below n_fixed stay, the rest are
            # renumbered (only their partition is observable)
            for h in [h for h in self.fixed if h >= self.n_fixed]:
                del handle[id(self.fixed.pop(h))]
            nxt = self.n_fixed
        for s, o in enumerate(self.stack):
            h = handle.get(id(o))
            if h is None:
                if count[id(o)] == 1 and not o.ann:
                    h = 0
                else:
                    h = handle[id(o)] = nxt
                    nxt += 1
                    b.omask[i, h] = _mask(o.ann)
            b.sobj[i, s] = h
        b.n_obj[i] = nxt
        b.n_atoms[i] = self.natoms
        b.sink[i] = _mask(self.sink)
        b.tflags[i] = self.tflags
        b.ymask[i] = _mask(self.ymask)


def _objects_full(lane: RefLane, cap: int) -> bool:
    """k_sym_step's object-table check before an instruction: after compaction the
    table holds the host's handles plus one per tracked object on the stack."""
    host = {id(o) for h, o in lane.fixed.items() if h < lane.n_fixed}
    env = {id(o) for o in lane.env.values()}
    live = {id(o) for o in lane.stack if o.tracked and id(o) not in host and id(o) not in env}
    return lane.n_fixed + len(live) + 4 > cap


def _word(b, i, slot) -> int:
    return limbs_to_word(b.stack[i, slot])


def _write_annot(b, i, at, atom, step, v0, v1, pc, opw, fent):
    q = b.rec[i]
    q[at], q[at + 1], q[at + 2] = MG_REC_ANNOT, atom, step
    q[at + 3: at + 11] = word_to_limbs(v0)
    q[at + MG_REC_HEADER: at + MG_REC_HEADER + 8] = word_to_limbs(v1)
    q[at + MG_REC_HEADER + 8] = pc
    q[at + MG_REC_HEADER + 9] = opw
    q[at + MG_REC_HEADER + 10] = fent          # the name the hook sees (before the instruction)


def _write_hook(b, i, at, words, step, pc, op):
    """MG_REC_HOOK: [kind][n][step][stack[-1]][stack[-2..-n]][pc][op][fent]."""
    q = b.rec[i]
    q[at], q[at + 1], q[at + 2] = MG_REC_HOOK, len(words), step
    q[at + 3: at + 11] = word_to_limbs(words[0])
    k = at + MG_REC_HEADER
    for w in words[1:]:
        q[k: k + 8] = word_to_limbs(w)
        k += 8
    q[k], q[k + 1], q[k + 2] = pc, op, b.fent[i]
    return k + 3 - at


def _snap(b, i):
    from mythril_amd.lanes import _ALL_FIELDS
    return {f: getattr(b, f)[i].copy() for f in _ALL_FIELDS}


def _restore(b, i, snap):
    for f, v in snap.items():
        getattr(b, f)[i] = v


def step_lane(oracle, ops: np.ndarray, b, i: int, lane: RefLane, actions, hook_mask, max_depth: int,
              acked: bool, loop_bound: int = 0, force=None) -> bool:
    """One instruction of taint lane i (its objects in `lane`), in k_sym_step's
    order: depth / end / trace and loop bound / hook / opcode escape, then the
    batch-safe hooks' checks, then the mutator.  Returns whether it executed;
    otherwise b.status[i] says why it stopped."""
    pc, sp = int(b.pc[i]), int(b.sp[i])
    steps0 = int(b.steps[i])
    flags0 = int(b.flags[i])
    snap = _snap(b, i)
    if acked or pc >= ops.size:
        # the host already ran this instruction's hooks: no device actions
        if acked and pc < ops.size and _objects_full(lane, b.shape.obj_cap):
            b.status[i], b.aux[i] = MG_ESCAPE, int(ops[pc]) | (MG_ESC_TAINT << 8)
            return False
        oracle.run(b, i, 1, hook_mask=hook_mask, max_steps=1, max_depth=max_depth, loop_bound=loop_bound)
        if int(b.steps[i]) != steps0 + 1:
            return False
        _objects(b, i, lane, int(ops[pc]), pc, sp, 0, None, None, snap)
        return True
    op = int(ops[pc])
    # probe: stop the lane right before the mutator (traced like any popped instruction)
    probe = list(int(x) for x in hook_mask)
    probe[op >> 6] |= 1 << (op & 63)
    oracle.run(b, i, 1, hook_mask=probe, max_steps=1, max_depth=max_depth, loop_bound=loop_bound)
    if int(b.status[i]) != MG_HOOK or (int(hook_mask[op >> 6]) >> (op & 63)) & 1:
        return False                    # depth, loop bound, trace full, or a real hook
    at_op = _snap(b, i)
    # an opcode the device escapes comes before the batch-safe hooks too
    b.status[i] = MG_RUNNING
    b.flags[i] = flags0 | MG_LANE_HOOK_ACK
    oracle.run(b, i, 1, hook_mask=(0, 0, 0, 0), max_steps=1, max_depth=max_depth, loop_bound=loop_bound)
    if int(b.status[i]) == MG_ESCAPE and (int(b.aux[i]) >> 8) == MG_ESC_OPCODE:
        b.flags[i] = flags0
        return False
    _restore(b, i, at_op)
    b.status[i], b.aux[i] = MG_RUNNING, 0
    tact = int(actions[op])
    if tact and force is not None and force[pc] == 1:
        b.status[i], b.aux[i] = MG_HOOK, op          # a cached issue address: the host's hooks
        return False
    if tact and force is not None and force[pc] == 2:
        tact = 0                                     # every module returns early there
    if not tact and _objects_full(lane, b.shape.obj_cap):
        b.status[i], b.aux[i] = MG_ESCAPE, op | (MG_ESC_TAINT << 8)
        return False
    yk, pre_k = (tact >> 12) & 15, tact & 15
    dk = (tact >> 16) & 15
    if yk and sp >= yk and (lane.stack[sp - yk].ann & lane.ymask):
        b.status[i], b.aux[i] = MG_HOOK, op
        return False
    # concrete lanes: an if-symbolic hook never has work; an if-annotation hook
    # has work when the host flagged the lane (tflags bit 1)
    if tact & MG_TAINT_IFLANE and lane.tflags & 2:
        b.status[i], b.aux[i] = MG_HOOK, op
        return False
    do_pre = pre_k != 0 and sp >= pre_k
    do_post = bool(tact & MG_TAINT_POST)
    if do_pre and tact & MG_TAINT_EXPCOND:
        base, ex = _word(b, i, sp - 1), (_word(b, i, sp - 2) if sp >= 2 else 0)
        if ex == 0 or base < 2:
            do_pre = False
    need = int(do_pre) + int(do_post)
    defer = dk != 0 and sp >= dk
    hook_words = MG_REC_HEADER + 8 * (dk - 1) + 3 if defer else 0
    if lane.natoms + need > 64 or _objects_full(lane, b.shape.obj_cap):
        b.status[i], b.aux[i] = MG_ESCAPE, op | (MG_ESC_TAINT << 8)
        return False
    if (need or defer) and int(b.rec_len[i]) + need * MG_REC_ANNOT_WORDS + hook_words > b.shape.rec_cap:
        b.status[i], b.aux[i] = MG_ESCAPE, op | (MG_ESC_RECORD << 8)
        return False
    pre_atom = post_atom = None
    rec0 = int(b.rec_len[i])
    fent0 = int(b.fent[i])
    if do_pre:
        _write_annot(b, i, rec0, lane.natoms, steps0, _word(b, i, sp - 1), _word(b, i, sp - 2) if sp >= 2 else 0,
                     pc, op, fent0)
        b.rec_len[i] = rec0 + MG_REC_ANNOT_WORDS
        pre_atom = lane.natoms
    if defer:
        at = int(b.rec_len[i])
        b.rec_len[i] = at + _write_hook(b, i, at, [_word(b, i, sp - 1 - j) for j in range(dk)], steps0, pc, op)
    b.flags[i] = flags0 | MG_LANE_HOOK_ACK          # run the mutator, not the trace again
    oracle.run(b, i, 1, hook_mask=(0, 0, 0, 0), max_steps=1, max_depth=max_depth, loop_bound=loop_bound)
    if int(b.steps[i]) != steps0 + 1:
        b.flags[i] = flags0
        b.rec_len[i] = rec0
        return False
    b.flags[i] = flags0
    if do_post:
        post_atom = lane.natoms + int(do_pre)
    _objects(b, i, lane, op, pc, sp, tact, pre_atom, post_atom, snap)
    if do_post:
        at = int(b.rec_len[i])
        nsp = int(b.sp[i])
        _write_annot(b, i, at, post_atom, steps0, _word(b, i, nsp - 1), _word(b, i, nsp - 2) if nsp >= 2 else 0,
                     pc, op | 0x100, fent0)
        b.rec_len[i] = at + MG_REC_ANNOT_WORDS
    for a in (pre_atom, post_atom):
        if a is not None:
            lane.natoms += 1
            if tact & MG_TAINT_YCLASS:
                lane.ymask.add(a)
    return True


def _objects(b, i, lane: RefLane, op, pc, sp0, tact, pre_atom, post_atom, snap):
    """The object effects of the executed instruction at pc (values before it in
    `snap`)."""
    st = lane.stack
    pre_k, sink_k = tact & 15, (tact >> 8) & 15
    if pre_atom is not None:
        st[sp0 - pre_k].ann.add(pre_atom)
        st[sp0 - pre_k].tracked = True
    if sink_k and sp0 >= sink_k:
        lane.sink |= st[sp0 - sink_k].ann
        lane.tflags |= 1
    before = [limbs_to_word(snap["stack"][s]) for s in range(max(0, sp0 - 3), sp0)][::-1]   # [-1], [-2], [-3]
    if 0x80 <= op <= 0x8F:                      # DUPn
        st[-(op - 0x7F)].tracked = True
        st.append(st[-(op - 0x7F)])
    elif 0x90 <= op <= 0x9F:                    # SWAPn
        n = op - 0x8F
        st[-1], st[-n - 1] = st[-n - 1], st[-1]
    else:
        nsp = int(b.sp[i])
        pushes = op not in NO_PUSH and not (0x60 <= op <= 0x7F and False)
        npop = sp0 + (1 if pushes else 0) - nsp
        popped = [st.pop() for _ in range(npop)]
        if pushes:
            if op in ENV_OPS:
                r = lane.env[ENV_OPS[op]]
            elif op in UNION2:
                r = Obj(popped[0].ann | popped[1].ann)
            elif op in ZERODIV:
                r = Obj() if before[1] == 0 else Obj(popped[0].ann | popped[1].ann)
            elif op in (0x08, 0x09):
                r = Obj(popped[0].ann | popped[1].ann | popped[2].ann)
            elif op in (0x15, 0x19):
                r = Obj(popped[0].ann)
            elif op == 0x1A:
                r = Obj(popped[1].ann) if before[0] < 32 else Obj()
            else:
                r = Obj()
            st.append(r)
    if post_atom is not None:
        st[-1].ann.add(post_atom)
        st[-1].tracked = True


def run_lane(oracle, ops, b, i: int, actions, hook_mask, max_steps: int, max_depth: int, horizon: int,
             loop_bound: int = 0, force=None) -> int:
    """k_sym_step on one taint lane: steps until it stops or its budget ends.
    Returns instructions executed."""
    if int(b.status[i]) != MG_RUNNING:
        return 0
    lane = RefLane(b, i)
    flags = int(b.flags[i])
    lane_max = min(max_steps, 1) if flags & MG_LANE_STEP1 else max_steps
    if horizon:
        s0 = int(b.steps[i])
        lane_max = min(lane_max, horizon - s0 if horizon > s0 else 0)
    executed = 0
    ack = bool(flags & MG_LANE_HOOK_ACK)
    while True:
        acked = ack and executed == 0
        if executed >= lane_max:
            # a budget pause: only the checks that precede it (depth, end, a hook,
            # whose pop is traced) can still stop the lane
            oracle.run(b, i, 1, hook_mask=hook_mask, max_steps=0, max_depth=max_depth, loop_bound=loop_bound)
            break
        if not step_lane(oracle, ops, b, i, lane, actions, hook_mask, max_depth, acked, loop_bound, force):
            break
        executed += 1
    if executed and ack:
        b.flags[i] = int(b.flags[i]) & ~MG_LANE_HOOK_ACK
    lane.write(b, i)
    return executed
