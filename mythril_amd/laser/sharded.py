"""Multi-transaction runs with the open world states sharded over the ranks
(SURVEY §8(e), config C5).

The reference's transaction loop (svm.py:239-275 ``_execute_transactions``)
starts one transaction per open world state, runs ``exec()`` and collects the
surviving world states as the next transaction's ``open_states``.  Here a
transaction round is one concrete ``MessageCallTransaction`` per (open world
state, calldata) pair — the symbolic calldata of the reference sampled by a
list of concrete calldatas — and the pairs of a round are partitioned over the
ranks, one process per GPU:

* the first round deals the (replicated) initial pairs round-robin, pair g to
  rank g % world; from then on every rank keeps the world states its own
  paths produced (no state ever crosses ranks — no data-path collective);
* the pairs a rank starts all run as lanes of ONE ``exec()``, i.e. one kernel-1
  batch per round per GPU;
* per round, the only exchange is a small all-gather: every rank's pair count
  (so transaction ids are the global pair positions, in rank-major order, and
  every rank's id counter advances by the global count — the re-sync §8(e)
  asks for, transaction_models.py:21-36) and the coverage bytes of every code
  (OR, coverage_plugin.py semantics) over RCCL (``dist.allgather_coverage``).

With one rank this is exactly the single-process loop.  The union over ranks
of the open world states equals the single-process run's (as a multiset of
account states; only the transaction ids differ, as §8(e) allows).
"""
from __future__ import annotations

from copy import copy
from typing import Dict, List, Optional, Sequence

import numpy as np

from .disassembly import Disassembly
from .transaction import MessageCallTransaction, _setup_global_state_for_execution, tx_id_manager


def _allgather_ints(x: int) -> List[int]:
    from .. import dist as mdist
    rank, world = mdist.rank_world()
    if world == 1:
        return [int(x)]
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(x)], dtype=torch.int64, device=mdist._device())
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [int(p.item()) for p in parts]


def _allgather_keys(keys: Sequence[str]) -> List[str]:
    from .. import dist as mdist
    rank, world = mdist.rank_world()
    if world == 1:
        return sorted(keys)
    import torch.distributed as dist
    out: List[Optional[List[str]]] = [None] * world
    dist.all_gather_object(out, sorted(keys))
    return sorted(set(k for part in out for k in (part or [])))


def exchange_coverage(laser_evm) -> Dict[str, np.ndarray]:
    """OR of every rank's coverage table ({bytecode: bytes}) into this rank's
    LaserEVM (it then reports the union, as one process covering every shard
    would); returns the union."""
    from .. import dist as mdist
    local = {code: np.asarray(bits, dtype=np.uint8) for code, (_, bits) in
             laser_evm.coverage().items()}
    union: Dict[str, np.ndarray] = {}
    for code in _allgather_keys(list(local)):
        n = _allgather_ints(local[code].size if code in local else 0)
        mine = np.zeros(max(n), dtype=np.uint8)
        if code in local:
            mine[:local[code].size] = local[code]
        union[code] = mdist.allgather_coverage(mine)
    laser_evm.merge_peer_coverage(union)
    return union


def _encode_model(model) -> list:
    """A Model as plain data (every internal ModelRef's assignment)."""
    from ..smt.program import ArrayInterp, FuncInterp
    out = []
    for ref in getattr(model, "raw", [model]):
        asg = {}
        for name, v in ref.assignment.items():
            if isinstance(v, ArrayInterp):
                asg[name] = ("A", v.default, dict(v.entries))
            elif isinstance(v, FuncInterp):
                asg[name] = ("F", v.else_value, dict(v.entries))
            else:
                asg[name] = int(v)
        out.append(asg)
    return out


def _decode_model(refs: list):
    from ..smt.program import ArrayInterp, FuncInterp
    from ..smt.solver import Model, ModelRef
    models = []
    for asg in refs:
        d = {}
        for name, v in asg.items():
            if isinstance(v, tuple) and v[0] == "A":
                d[name] = ArrayInterp(v[1], v[2])
            elif isinstance(v, tuple) and v[0] == "F":
                d[name] = FuncInterp(v[1], v[2])
            else:
                d[name] = v
        models.append(ModelRef(d))
    return Model(models)


def exchange_models(model_cache=None) -> int:
    """the satisfying models every rank found since the last
    exchange (z3 fallback answers cached by get_model, support/model.py:76-78)
    join every other rank's candidate pool — kernel 2's ModelCache — in rank
    order, each with count 1 as a fresh backend model gets.  One all-gather per
    transaction round; returns the number of peer models received."""
    from .. import dist as mdist
    from ..smt import solver
    cache = model_cache or solver.model_cache
    rank, world = mdist.rank_world()
    mine = [_encode_model(m) for m in cache.take_fresh()]
    if world == 1:
        return 0
    import torch.distributed as dist
    parts: List[Optional[list]] = [None] * world
    dist.all_gather_object(parts, mine)
    got = 0
    for r, models in enumerate(parts):
        if r == rank:
            continue
        for enc in models or []:
            cache.put(_decode_model(enc), 1, peer=True)
            got += 1
    return got


def execute_message_calls(laser_evm, callee_address, caller_address, origin_address,
                          datas: Sequence[bytes], gas_limit, gas_price, value, code=None,
                          track_gas: bool = False, exchange_cov: bool = True):
    """One transaction round: a MessageCallTransaction for every (open world
    state, calldata) pair this rank owns, all run by one ``laser_evm.exec``.
    Returns the final states when ``track_gas`` (this rank's paths)."""
    from .. import dist as mdist
    rank, world = mdist.rank_world()
    open_states = laser_evm.open_states[:]
    del laser_evm.open_states[:]
    if getattr(laser_evm, "use_reachability_check", False):
        # svm.py:244-249: a transaction starts only from open states whose path
        # constraints are possible (kernel-2 quick-sat, then the SMT backend)
        from ..smt.solver import Constraints
        open_states = [ws for ws in open_states if Constraints(ws.constraints).is_possible()]
    local = [(ws, d) for ws in open_states for d in datas]
    if world > 1 and not getattr(laser_evm, "_sharded", False):
        # replicated start: deal pair g to rank g % world
        total = len(local)
        mine = [(g, p) for g, p in enumerate(local) if g % world == rank]
    else:
        counts = _allgather_ints(len(local))
        off = sum(counts[:rank])
        total = sum(counts)
        mine = [(off + j, p) for j, p in enumerate(local)]
    base = tx_id_manager._next_transaction_id
    for g, (ws, data) in mine:
        # every calldata of a world state starts from its own copy of it
        world_state = ws if len(datas) == 1 else copy(ws)
        bytecode = code or world_state[callee_address].code.bytecode
        tx = MessageCallTransaction(
            world_state=world_state,
            identifier=str(base + g + 1),
            gas_price=gas_price,
            gas_limit=gas_limit,
            origin=origin_address,
            code=Disassembly(bytecode),
            caller=caller_address,
            callee_account=world_state[callee_address],
            call_data=data,
            call_value=value,
        )
        _setup_global_state_for_execution(laser_evm, tx)
    tx_id_manager.set_counter(base + total)
    laser_evm._sharded = world > 1
    final = laser_evm.exec(track_gas=track_gas)
    if exchange_cov and world > 1 and laser_evm.record_coverage:
        exchange_coverage(laser_evm)
    if world > 1:
        exchange_models()
    return final


def open_state_counts(laser_evm) -> List[int]:
    """Every rank's number of open world states (rank order)."""
    return _allgather_ints(len(laser_evm.open_states))
