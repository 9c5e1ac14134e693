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
