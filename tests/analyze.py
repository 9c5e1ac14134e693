"""``myth analyze -f <creation code> -t N -m <module> --no-onchain-data`` on the
batched core -- test infrastructure for the integration rows of
tests/integration_tests/analysis_tests.py:9-54 (tests/golden/integration.json).

Mirrors analysis/symbolic.py:82-200 (SymExecWrapper) for the parts the rows
use: the creator and attacker accounts, BFS with BoundedLoopsStrategy(3),
max depth 128, the module's pre/post hooks, a symbolic creation then N symbolic
message calls (svm.py:142-212 sym_exec).  What stands in for the reference's
own code (none of it importable here):
* escapes (CALL*, SELFDESTRUCT, BALANCE, ...) are stepped by the CPU
  restatement tests/symref.py in its escape-handler form;
* modules are the restatements in tests/refmodules.py;
* issue confirmation is SAT-only (mythril_amd.smt.search.SatSearchBackend:
  kernel 2 over the model cache, the witness seeds and a guided candidate
  search) -- it returns a model or "unknown", never "unsat", so an issue the
  reference confirms can at worst stay unconfirmed here (counted)."""
from __future__ import annotations

import time

import refmodules
import symref
from mythril_amd import workloads
from mythril_amd.laser import Account, BoundedLoopsStrategy, BreadthFirstSearchStrategy, LaserEVM, WorldState
from mythril_amd.laser import svm as svm_mod
from mythril_amd.laser.transaction import ACTORS, tx_id_manager
from mythril_amd.laser.witness import WitnessSeeds
from mythril_amd.smt import solver
from mythril_amd.smt.exponent_manager import exponent_function_manager
from mythril_amd.smt.keccak_manager import keccak_function_manager


def analyze(name: str, module: str, tx_count: int, device, k2, n_seeds: int = 256, search=True):
    """Run the analysis; returns (issues, info)."""
    from mythril_amd.smt.search import SatSearchBackend
    keccak_function_manager.reset()
    exponent_function_manager.reset()
    tx_id_manager.restart_counter()
    refmodules.CONFIRMATIONS.update(sat=0, unknown=0)
    code = workloads.bytecode(name)
    mod = getattr(refmodules, module)()
    saved = (solver.model_cache, solver.solver_backend, svm_mod.check_potential_issues)
    mc = solver.ModelCache(device=k2)
    mc.seed_source = WitnessSeeds([code], n=n_seeds, balance_names=["balance"])
    solver.model_cache = mc
    backend = SatSearchBackend(mc, search=search)
    solver.set_solver_backend(backend)
    svm_mod.check_potential_issues = refmodules.check_potential_issues
    try:
        laser = LaserEVM(device=device, strategy=BreadthFirstSearchStrategy, max_depth=128,
                         execution_timeout=86400, create_timeout=10, transaction_count=tx_count,
                         requires_statespace=False, escape_handler=symref.Engine(signals=True).step)
        laser.unknown_forks = "keep"
        laser.extend_strategy(BoundedLoopsStrategy, loop_bound=3)
        laser.register_hooks("pre", refmodules.hooks_of([mod], "pre"))
        laser.register_hooks("post", refmodules.hooks_of([mod], "post"))
        ws = WorldState()
        for actor in ("CREATOR", "ATTACKER"):
            ws.put_account(Account(ACTORS[actor], contract_name=None))
        t0 = time.perf_counter()
        laser.sym_exec(world_state=ws, creation_code=code, contract_name="MAIN")
        wall = time.perf_counter() - t0
        info = {"wall_s": wall, "lane_steps": laser.lane_steps, "launches": laser.launches,
                "forks": laser.forks, "fork_filter": dict(laser.fork_stats),
                "escapes_dropped": laser.escapes_dropped, "confirmations": dict(refmodules.CONFIRMATIONS),
                "cache": dict(mc.stats), "search": dict(backend.stats),
                "kernel2_launches": mc.launches, "device_evals": mc.device_evals}
        return list(mod.issues), info
    finally:
        solver.model_cache, _, svm_mod.check_potential_issues = saved
        solver.set_solver_backend(saved[1])
