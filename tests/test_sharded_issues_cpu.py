"""Issues of a sharded analysis merged across ranks (mythril_amd/
laser/sharded.py merge_issues), on CPU: gloo ranks, the C oracles as kernels 1
and 2, the restated modules and the SAT-only confirmation of tests/analyze.py.

Every rank runs the symbolic creation (replicated), then the message-call
rounds with the open states sharded and rebalanced
(execute_symbolic_transactions); each rank's modules hold the issues its paths
filed.  After merge_issues every rank must hold the issue set of the
single-process run -- (SWC id, address, function, title) of each issue, the
reference's report rows -- de-duplicated by the modules' cache key: the
creation's issues, which every rank files, appear once.  The exchanges travel
as u32 value streams (no pickled objects), checked by a round trip here."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

CASES = [("exceptions_0.8.0.sol.o", "Exceptions", 2), ("extcall.sol.o", "Exceptions", 1)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(name, module, tx_count, sigdir):
    import refmodules
    import symref
    from fnames import signature_db
    from pathlib import Path
    from mythril_amd import workloads
    from mythril_amd.laser import (Account, BoundedLoopsStrategy, BreadthFirstSearchStrategy, LaserEVM,
                                   WorldState, execute_symbolic_contract_creation)
    from mythril_amd.laser import svm as svm_mod
    from mythril_amd.laser.disassembly import SignatureDB
    from mythril_amd.laser.sharded import execute_symbolic_transactions, merge_issues
    from mythril_amd.laser.transaction import ACTORS, tx_id_manager
    from mythril_amd.laser.witness import WitnessSeeds
    from mythril_amd.smt import solver
    from mythril_amd.smt.exponent_manager import exponent_function_manager
    from mythril_amd.smt.keccak_manager import keccak_function_manager
    from mythril_amd.smt.search import SatSearchBackend
    from oracle_device import OracleDevice, OracleK2

    signature_db(Path(sigdir))
    os.environ["MYTHRIL_DIR"] = sigdir
    SignatureDB._reset()
    keccak_function_manager.reset()
    exponent_function_manager.reset()
    tx_id_manager.restart_counter()
    code = workloads.bytecode(name)
    mc = solver.ModelCache(device=OracleK2())
    mc.seed_source = WitnessSeeds([code], n=256, balance_names=["balance"])
    solver.model_cache = mc
    solver.set_solver_backend(SatSearchBackend(mc))
    svm_mod.check_potential_issues = refmodules.check_potential_issues
    mods = refmodules.detection_modules([module])
    vm = LaserEVM(device=OracleDevice(), strategy=BreadthFirstSearchStrategy, max_depth=128,
                  execution_timeout=86400, transaction_count=tx_count, requires_statespace=False,
                  escape_handler=symref.Engine(signals=True).step)
    vm.unknown_forks = "keep"
    vm.extend_strategy(BoundedLoopsStrategy, loop_bound=3)
    refmodules.MutationPruner().initialize(vm)
    vm.register_hooks("pre", refmodules.hooks_of(mods, "pre"))
    vm.register_hooks("post", refmodules.hooks_of(mods, "post"))
    ws = WorldState()
    for actor in ("CREATOR", "ATTACKER"):
        ws.put_account(Account(ACTORS[actor], contract_name=None))
    created = execute_symbolic_contract_creation(vm, code, "MAIN", world_state=ws)
    execute_symbolic_transactions(vm, created.address)
    unmerged = sorted({i.key() for m in mods for i in m.issues})
    before = len(unmerged)
    merged = merge_issues(mods, refmodules.Issue)
    return sorted(i.key() for m in mods for i in m.issues), merged, before, unmerged


def _worker(rank, world, port, out, case, sigdir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out[rank] = _run(*case, sigdir)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_sharded_issue_sets_equal_single_process(case, tmp_path):
    single, n, _, unmerged = _run(*case, str(tmp_path / "sig"))
    # the one-process baseline is the run's own issue set, not a merge of it
    assert single == unmerged and n == len(single) and single
    for world in (2, 3):
        port = _free_port()
        with mp.Manager() as m:
            out = m.dict()
            mp.spawn(_worker, args=(world, port, out, case, str(tmp_path / "sig")), nprocs=world, join=True)
            res = [out[r] for r in range(world)]
        for issues, merged, _, _ in res:
            assert issues == single and merged == len(single), (world, issues, single)
        if case[0] == "extcall.sol.o":
            # the constructor's issue: every rank filed it, the merge keeps one
            assert all(before == len(single) for _, _, before, _ in res)
        else:
            # the message calls' issues: some rank filed fewer than the merged set
            assert min(before for _, _, before, _ in res) < len(single)


def test_value_stream_round_trips():
    from mythril_amd.laser.sharded import _Words, _get_value, _values_to_words
    v = (None, True, False, 0, -5, (1 << 300) + 7, "MAIN", b"\x00\x01", [1, (2, "x")],
         {"steps": [{"input": "0xab", "value": "0x0"}], 3: None}, 0.125, -1e300, 12.3456789)
    assert _get_value(_Words(_values_to_words(v))) == v


class _RefIssue:
    """The reference's Issue shape (report.py:26-72): bytecode_hash, no
    bytecode, a float discovery_time."""

    def __init__(self, address, code_hash, title, t):
        self.address, self.bytecode_hash, self.title = address, code_hash, title
        self.swc_id, self.function, self.contract = "106", "kill()", "MAIN"
        self.discovery_time = t
        self.transaction_sequence = {"steps": [{"input": "0x41c0e1b5", "value": "0x0"}]}
        self.source_location = None


class _RefModule:
    """base.py:55-70: caches (address, bytecode_hash)."""
    auto_cache = True

    def __init__(self, issues):
        self.issues, self.cache = list(issues), set()

    def update_cache(self, issues=None):
        for issue in issues or self.issues:
            self.cache.add((issue.address, issue.bytecode_hash))


def test_merge_keys_reference_issues_on_the_code_hash():
    """two contracts at the same address are two issues; the cache
    gets the module's own (address, bytecode_hash) keys; floats survive."""
    from mythril_amd.laser.sharded import merge_issues
    m = _RefModule([_RefIssue(146, "0xaa", "Unprotected Selfdestruct", 0.25),
                    _RefIssue(146, "0xbb", "Unprotected Selfdestruct", 0.5),
                    _RefIssue(146, "0xaa", "Unprotected Selfdestruct", 0.75)])
    assert merge_issues([m], _RefIssue) == 2
    assert m.cache == {(146, "0xaa"), (146, "0xbb")}
    assert [i.discovery_time for i in m.issues] == [0.25, 0.5]
    assert m.issues[0].transaction_sequence["steps"][0]["input"] == "0x41c0e1b5"


def test_merge_refuses_an_attribute_it_cannot_send():
    from mythril_amd.laser.sharded import merge_issues
    i = _RefIssue(1, "0xaa", "t", 0.0)
    i.detector = object()
    with pytest.raises(TypeError, match="detector"):
        merge_issues([_RefModule([i])], _RefIssue)
