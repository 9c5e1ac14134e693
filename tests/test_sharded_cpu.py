"""Transaction rounds with open world states sharded over ranks (SURVEY §8(e),
C5; mythril_amd/laser/sharded.py), on CPU: gloo ranks, the host LASER mirror
over the oracle-backed device (tests/oracle_device.py).

Checks, against the single-process run of the same rounds:
* the union over ranks of the open world states is the same multiset of
  callee states (storage + balance);
* every rank's coverage after the exchange is the single-process coverage;
* every rank's transaction-id counter equals the single-process counter, and
  the ids handed out across ranks are exactly 1..total (no duplicates).
"""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from mythril_amd import workloads

CALLEE = 0x0901D12EBE1B195E5AA8748E62BD7734AE19B51F
ATTACKER = workloads.ATTACKER


def _word(x: int) -> bytes:
    return int(x).to_bytes(32, "big")


DATAS = [
    bytes.fromhex("18160ddd"),                                   # totalSupply()
    bytes.fromhex("70a08231") + _word(ATTACKER),                 # balanceOf(attacker)
    bytes.fromhex("a3210e87") + _word(0x1234) + _word(1),        # sendeth(0x1234, 1)
    bytes.fromhex("a3210e87") + _word(ATTACKER) + _word(7),      # sendeth(attacker, 7)
    bytes.fromhex("deadbeef"),                                   # no such function
]
ROUNDS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rounds():
    """Run ROUNDS transaction rounds in this process (rank from torch.distributed
    if initialised); returns (fingerprints, coverage, counter, ids, lane_steps)."""
    from mythril_amd.laser import (Account, Disassembly, InstructionCoveragePlugin, LaserEVM,
                                   WorldState, tx_id_manager)
    from mythril_amd.laser.sharded import execute_message_calls
    from mythril_amd.smt import solver
    from oracle_device import OracleDevice, OracleK2

    # the reachability filter's queries (each round's transaction appends its
    # UGE(balances[sender], value) conjunct) run on the oracle's kernel 2
    saved = solver.model_cache
    solver.model_cache = solver.ModelCache(device=OracleK2())
    solver.get_model.cache_clear()
    try:
        return _rounds_body(execute_message_calls, OracleDevice())
    finally:
        solver.model_cache = saved
        solver.get_model.cache_clear()


def _rounds_body(execute_message_calls, device):
    from mythril_amd.laser import (Account, Disassembly, InstructionCoveragePlugin, LaserEVM,
                                   WorldState, tx_id_manager)
    tx_id_manager.restart_counter()
    ws = WorldState()
    acct = Account(CALLEE, concrete_storage=True)
    acct.code = Disassembly(workloads.bytecode("overflow.sol.o").hex())
    ws.put_account(acct)
    vm = LaserEVM(requires_statespace=False, device=device)
    cov = InstructionCoveragePlugin()
    cov.initialize(vm)
    vm.open_states = [ws]
    ids = []
    for _ in range(ROUNDS):
        execute_message_calls(vm, CALLEE, ATTACKER, ATTACKER, DATAS, gas_limit=8_000_000,
                              gas_price=0, value=0)
        for s in vm.open_states:
            ids.append(s.transaction_sequence[-1].id)
    prints = sorted((tuple(sorted(s[CALLEE].storage.items())), str(s[CALLEE].balance().raw))
                    for s in vm.open_states)
    table = {k: list(v[1]) for k, v in vm.coverage().items()}
    return prints, table, tx_id_manager._next_transaction_id, ids, vm.lane_steps


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out[rank] = _rounds()
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def single():
    return _rounds()


def test_single_process_rounds_fork_the_open_states(single):
    prints, table, counter, ids, steps = single
    # round r starts |open| x |DATAS| transactions; reverting calls leave no open state
    assert len(prints) > len(DATAS) and steps > 0
    assert counter >= len(prints) and len(set(ids[-len(prints):])) == len(prints)
    assert any(any(bits) for bits in table.values())


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_rounds_equal_single_process(single, world):
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = [out[r] for r in range(world)]
    prints, table, counter, _, steps = single
    union = sorted(p for r in res for p in r[0])
    assert union == prints
    for r in res:
        assert r[1] == table             # coverage after the all-gather = 1-process coverage
        assert r[2] == counter           # re-synchronised transaction-id counters
    # ids of the final open states across ranks: no duplicates
    last = [i for r in res for i in r[3][-len(r[0]):]] if all(r[0] for r in res) else []
    assert len(last) == len(set(last))
    assert sum(r[4] for r in res) == steps
    # every rank did part of the work
    assert all(r[4] > 0 for r in res)
