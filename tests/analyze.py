"""``myth analyze`` / ``myth safe-functions`` on the batched core -- test
infrastructure for the reference's integration rows
(tests/integration_tests/analysis_tests.py:9-82, test_safe_functions.py:26-51;
tests/golden/integration.json) and the C1 stand-in.

Mirrors analysis/symbolic.py:47-200 (SymExecWrapper) and cli.py:733-803 for the
parts the rows use: the creator and attacker accounts, the strategy (BFS, or
``--strategy delayed``: DelayConstraintStrategy) with BoundedLoopsStrategy(3),
max depth 128, the MutationPruner plugin, the modules' pre/post hooks, then
either a symbolic creation and N symbolic message calls (``-f code``) or N
message calls into the runtime code at address 0 with symbolic storage
(``--bin-runtime -f code``, util.get_indexed_address(0)).  What stands in for
the reference's own code (none of it importable here):
* escapes (CALL*, SELFDESTRUCT, BALANCE, ...) are stepped by the CPU
  restatement tests/symref.py in its escape-handler form;
* modules (all fourteen, loader order) and the mutation pruner are the
  restatements in tests/refmodules.py;
* issue confirmation is SAT-only (mythril_amd.smt.search.SatSearchBackend:
  kernel 2 over the model cache, the witness seeds and a guided candidate
  search) -- it returns a model or "unknown", never "unsat", so an issue the
  reference confirms can at worst stay unconfirmed here (counted).
Not restated: the dependency pruner (on by default for ``analyze``, off for
``safe-functions``): it only drops states of later transactions that read no
storage the earlier ones wrote, and the rows' issue sets do not depend on it."""
from __future__ import annotations

import time
from typing import Optional, Sequence

import refmodules
import symref
from mythril_amd import workloads
from mythril_amd.laser import Account, BoundedLoopsStrategy, BreadthFirstSearchStrategy, LaserEVM, WorldState
from mythril_amd.laser import svm as svm_mod
from mythril_amd.laser.disassembly import Disassembly
from mythril_amd.laser.strategy import DelayConstraintStrategy
from mythril_amd.laser.transaction import ACTORS, tx_id_manager
from mythril_amd.laser.witness import WitnessSeeds
from mythril_amd.smt import solver
from mythril_amd.smt.exponent_manager import exponent_function_manager
from mythril_amd.smt.keccak_manager import keccak_function_manager


def analyze(name: str, modules, tx_count: int, device, k2, n_seeds: int = 256, search=True,
            strategy: str = "bfs", runtime: bool = False, code: Optional[bytes] = None,
            mutation_pruner: bool = True, exact: bool = True, exact_ms: int = 60000,
            statespace: bool = False):
    """Run one analysis; returns (report issues, info).  `modules`: a module
    name, a list of names, or None (all fourteen).  `exact`: the queries the
    SAT search leaves open go to the exact procedure (mythril_amd.smt.exact),
    so fork filters and confirmations prune on unsat and on a budget timeout
    exactly as the reference's is_possible / get_model do; without it they
    stay "unknown" and the paths are kept (the prefilter-only mode).
    `statespace`: requires_statespace, as SymExecWrapper sets it for POST
    modules and graphs (symbolic.py:110-113): every state stepped one
    instruction at a time and the graph built."""
    from mythril_amd.smt.search import SatSearchBackend
    keccak_function_manager.reset()
    exponent_function_manager.reset()
    tx_id_manager.restart_counter()
    refmodules.CONFIRMATIONS.update(sat=0, unknown=0, timeout=0, unsat=0)
    code = workloads.bytecode(name) if code is None else code
    white = [modules] if isinstance(modules, str) else modules
    mods = refmodules.detection_modules(white)
    saved = (solver.model_cache, solver.solver_backend, svm_mod.check_potential_issues)
    mc = solver.ModelCache(device=k2)
    mc.seed_source = WitnessSeeds([code], n=n_seeds, balance_names=["balance"])
    solver.model_cache = mc
    if exact:
        from mythril_amd.smt.exact import ExactSolver
        backend = SatSearchBackend(mc, search=search, exact=ExactSolver(max_ms=exact_ms), exact_ms=exact_ms)
    else:
        backend = SatSearchBackend(mc, search=search)
    solver.set_solver_backend(backend)
    svm_mod.check_potential_issues = refmodules.check_potential_issues
    strat = {"bfs": BreadthFirstSearchStrategy, "delayed": DelayConstraintStrategy}[strategy]
    try:
        laser = LaserEVM(device=device, strategy=strat, max_depth=128,
                         execution_timeout=86400, create_timeout=10, transaction_count=tx_count,
                         requires_statespace=statespace, escape_handler=symref.Engine(signals=True).step)
        if strategy == "delayed":
            laser.strategy.model_cache._device = k2
            if not exact:
                laser.strategy.unknown = "keep"      # as the fork filters' unknown answers
        if not exact:
            laser.unknown_forks = "keep"
        laser.extend_strategy(BoundedLoopsStrategy, loop_bound=3)
        if mutation_pruner:
            refmodules.MutationPruner().initialize(laser)
        laser.register_hooks("pre", refmodules.hooks_of(mods, "pre"))
        laser.register_hooks("post", refmodules.hooks_of(mods, "post"))
        ws = WorldState()
        t0 = time.perf_counter()
        if runtime:
            # symbolic.py:117-120, 156-167: the attacker, and the code at the
            # indexed address 0 with symbolic storage
            ws.put_account(Account(ACTORS["ATTACKER"], contract_name=None))
            ws.put_account(Account(0, code=Disassembly(code), contract_name="MAIN", balances=ws.balances,
                                   concrete_storage=False))
            laser.sym_exec(world_state=ws, target_address=0)
        else:
            for actor in ("CREATOR", "ATTACKER"):
                ws.put_account(Account(ACTORS[actor], contract_name=None))
            laser.sym_exec(world_state=ws, creation_code=code, contract_name="MAIN")
        wall = time.perf_counter() - t0
        issues = refmodules.report_issues(mods)
        info = {"wall_s": wall, "lane_steps": laser.lane_steps, "launches": laser.launches,
                "forks": laser.forks, "fork_filter": dict(laser.fork_stats),
                "escapes_dropped": laser.escapes_dropped, "confirmations": dict(refmodules.CONFIRMATIONS),
                "cache": dict(mc.stats), "search": dict(backend.stats),
                "exact": dict(backend.exact.stats) if backend.exact is not None else None,
                "kernel2_launches": mc.launches, "device_evals": mc.device_evals,
                "device_ms": laser.device_ms, "k2_ms": mc.device_ms, "modules": [type(m).__name__ for m in mods]}
        return issues, info
    finally:
        solver.model_cache, _, svm_mod.check_potential_issues = saved
        solver.set_solver_backend(saved[1])


def safe_functions(name: str, device, k2, code: Optional[bytes] = None, **kw):
    """cli.py:788-803 + print_function_report (cli.py:733-753): one symbolic
    transaction into the runtime code with every module; the functions of the
    dispatcher table no issue was filed in.  Returns (safe names, issues, info)."""
    code = workloads.bytecode(name) if code is None else code
    issues, info = analyze(name, None, 1, device, k2, runtime=True, code=code, **kw)
    functions = set(Disassembly(code).address_to_function_name.values())
    for issue in issues:
        if issue.contract == "MAIN":
            functions.discard(issue.function)
    return sorted(functions), issues, info


def issue_table(issues: Sequence) -> list:
    """(SWC, address, function, title) rows, sorted: what the rows compare."""
    return sorted(i.key() for i in issues)
