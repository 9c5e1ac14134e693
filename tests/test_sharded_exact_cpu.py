"""bench.py's symbolic_tx field with the exact procedure behind kernel 2, sharded
over 2 gloo ranks (laser/sharded.py execute_symbolic_transactions: open states
rebalanced at every transaction boundary), against one process running the
same replicas -- the path the driver's multi-GPU bench takes.  On CPU with
the oracle-backed device.  Summed over the ranks, the forks, the pruned forks,
the unsat answers, the transaction ends and the open states equal the
single-process run: each rank's own exact procedure prunes what one process
prunes (the sat answers may differ, since each rank's model cache answers
different queries first)."""
import json
import os
import socket

import torch.distributed as dist
import torch.multiprocessing as mp

NAME = "overflow.sol.o"


def _dev():
    from oracle_device import OracleDevice, OracleK2

    class _Both(OracleDevice):
        def __init__(self):
            super().__init__()
            self._k2 = OracleK2()

        def eval(self, prog, pool):
            return self._k2.eval(prog, pool)

        def eval_bits(self, prog, pool):
            return self._k2.eval_bits(prog, pool)
    return _Both()


def _run(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import symref
        bench.SYMBOLIC_TX_CODES = (NAME,)
        r = bench.run_symbolic_tx(_dev(), 2 // world, 2, 256, symref.Engine(signals=True).step)
        c = r["contracts"][NAME]
        with open(f"{out}.{rank}.json", "w") as f:
            json.dump({"forks": c["forks"], "pruned": c["fork_filter"]["pruned"], "open": c["open_states"],
                       "unsat": c["exact"]["exact_unsat"], "timeout": c["exact"]["exact_timeout"],
                       "ends": c["tx_ends"]}, f)
    finally:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_sharded_symbolic_tx_with_the_exact_procedure_matches_one_process(tmp_path, monkeypatch):
    for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE"):
        monkeypatch.setenv(k, os.environ.get(k, ""))       # restored after the in-process leg
    one = tmp_path / "one"
    _run(0, 1, _port(), str(one))
    two = tmp_path / "two"
    mp.spawn(_run, args=(2, _port(), str(two)), nprocs=2)
    a = json.loads((tmp_path / "one.0.json").read_text())
    parts = [json.loads((tmp_path / f"two.{r}.json").read_text()) for r in range(2)]
    for k in ("forks", "pruned", "open", "unsat", "timeout"):
        assert sum(p[k] for p in parts) == a[k], (k, parts, a)
    for k in ("return_or_stop", "revert"):
        assert sum(p["ends"][k] for p in parts) == a["ends"][k]
    assert a["pruned"] > 0 and a["unsat"] > 0 and all(p["forks"] for p in parts)
