"""bench.run_myth_analyze (the C3-shaped field: ``myth analyze -f <code> -t 2``
with every module over the 18 reference contracts) on the CPU oracle device:
the field's structure, the per-contract issue tables (the integration rows'
issues among them), the CPU comparator's agreement, and the dealing of
contracts over gloo ranks."""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import bench  # noqa: E402
from mythril_amd import workloads  # noqa: E402
from oracle_device import OracleDevice, OracleK2  # noqa: E402

NAMES = ["suicide.sol.o", "origin.sol.o", "exceptions_0.8.0.sol.o"]


class _Both(OracleDevice):
    """Lanes and kernel 2 on one object, as GpuDevice has them."""

    def __init__(self):
        super().__init__()
        self.k2 = OracleK2()

    def __getattr__(self, name):
        return getattr(self.__dict__["k2"], name)


def test_the_eighteen_reference_contracts_are_the_field():
    assert len(workloads.bytecode_names()) == 18


def test_myth_analyze_field_on_the_oracle_device():
    out = bench.run_myth_analyze(_Both(), 2, names=NAMES)
    assert out["contracts_analysed"] == 3 and sorted(out["contracts"]) == sorted(NAMES)
    rows = out["contracts"]
    assert rows["suicide.sol.o"]["issues"] == [["106", 146, "constructor", "Unprotected Selfdestruct"]]
    assert [r[:3] for r in rows["exceptions_0.8.0.sol.o"]["issues"]] == \
        [["110", 186, "assert1()"], ["110", 186, "fail()"]]
    assert out["totals"]["escapes_dropped"] == 0
    assert out["totals"]["issues"] == sum(len(r["issues"]) for r in rows.values())
    cpu = out["cpu_baseline"]
    assert cpu["issue_sets_match"] and cpu["unit"] == "contracts/s" and cpu["cores"] >= 1
    assert out["contracts_per_s"] > 0


def _rank_worker(rank, world, port, out):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = bench.run_myth_analyze(_Both(), 1, names=NAMES)
        out[rank] = {"mine": sorted(res["contracts"]), "totals": res["totals"], "ranks": res["ranks"],
                     "job_wall": res["job_wall_s"], "cpu": "cpu_baseline" in res}
    finally:
        dist.destroy_process_group()


def test_myth_analyze_deals_contracts_over_ranks():
    """With N ranks each analyses contracts rank::N (total work fixed); the job
    wall is the slowest rank's; the CPU comparator runs only at N=1."""
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
    assert r0["mine"] == ["exceptions_0.8.0.sol.o", "suicide.sol.o"] and r1["mine"] == ["origin.sol.o"]
    assert r0["ranks"] == r1["ranks"] == 2
    assert r0["job_wall"] == r1["job_wall"] == max(r0["totals"]["wall_s"], r1["totals"]["wall_s"])
    assert not r0["cpu"] and not r1["cpu"]
