"""bench.run_analyses (the 18-contract `-t 2` field) on the CPU oracle device:
the field's structure, and that a myth-style analysis with the filters on keeps
every path no candidate refutes (no SMT backend: nothing is pruned)."""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import bench  # noqa: E402
import symref  # noqa: E402
from mythril_amd import workloads  # noqa: E402
from oracle_device import OracleDevice, OracleK2  # noqa: E402


class _Both(OracleDevice):
    """Lanes and kernel 2 on one object, as GpuDevice has them."""

    def __init__(self):
        super().__init__()
        self.k2 = OracleK2()

    def __getattr__(self, name):
        return getattr(self.__dict__["k2"], name)


def test_the_eighteen_reference_contracts_are_the_field():
    assert len(workloads.bytecode_names()) == 18


def test_analyses_field_on_the_oracle_device():
    names = ["suicide.sol.o", "origin.sol.o", "calls.sol.o"]
    out = bench.run_analyses(_Both(), 2, 256, escape_handler=symref.Engine(signals=True).step, names=names)
    assert out["contracts_analysed"] == 3 and sorted(out["contracts"]) == sorted(names)
    tot = out["totals"]
    assert tot["queries"] > 0 and tot["answered"] + tot["unknown"] == tot["queries"]
    assert tot["pruned"] == 0 and tot["escapes_dropped"] == 0
    assert out["prefilter_hit_rate"] is not None and 0 <= out["prefilter_hit_rate"] <= 1
    assert out["contracts"]["calls.sol.o"]["open_states"] >= 1


def _rank_worker(rank, world, port, out):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        names = ["suicide.sol.o", "origin.sol.o", "calls.sol.o"]
        res = bench.run_analyses(_Both(), 2, 128, escape_handler=symref.Engine(signals=True).step, names=names)
        out[rank] = {"mine": sorted(res["contracts"]), "totals": res["totals"], "ranks": res["ranks"],
                     "job_wall": res["job_wall_s"], "rate": res["job_constraint_evals_per_s_wall"],
                     "hit": res["prefilter_hit_rate"]}
    finally:
        dist.destroy_process_group()


def test_analyses_field_deals_contracts_over_ranks():
    """With N ranks each analyses contracts rank::N (total work fixed); the job
    figures sum the ranks' work over the slowest rank's wall time."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rank_worker, args=(2, port, out), nprocs=2, join=True)
        r0, r1 = dict(out[0]), dict(out[1])
    assert r0["mine"] == ["calls.sol.o", "suicide.sol.o"] and r1["mine"] == ["origin.sol.o"]
    assert r0["ranks"] == r1["ranks"] == 2
    assert r0["job_wall"] == r1["job_wall"] == max(r0["totals"]["wall_s"], r1["totals"]["wall_s"])
    evals = r0["totals"]["constraint_evals"] + r1["totals"]["constraint_evals"]
    assert abs(r0["rate"] - evals / r0["job_wall"]) < 1e-6 * max(evals, 1)
    q = r0["totals"]["queries"] + r1["totals"]["queries"]
    a = r0["totals"]["answered"] + r1["totals"]["answered"]
    assert r0["hit"] == r1["hit"] == a / q
