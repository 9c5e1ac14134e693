"""The symbolic half of the boundary on an MI355X: a reference-shaped
symbolic GlobalState (tests/refshapes.py, z3 terms from tests/fakez3.py) is
packed with bridge.pack_global_state, run by the batched LaserEVM as symbolic
lanes on kernel 1 (symbolic calldata, sender, storage with a symbolic Store,
a symbolic memory byte, a path constraint), and every path ends exactly as
the CPU restatement (tests/symref.py) ends the same packed state; the final
states write back into reference-shaped objects (bridge.unpack_global_state)
whose z3 terms lower to the device's expressions node for node."""
from collections import Counter
from copy import copy

import pytest

import fakez3 as z
import refshapes as R
import symcases
import symref
from mythril_amd import bridge
from mythril_amd.device import GpuDevice
from mythril_amd.laser import BreadthFirstSearchStrategy, LaserEVM
from mythril_amd.smt import solver
from test_bridge import _symbolic_ref_state

pytestmark = pytest.mark.gpu


def test_packed_symbolic_state_runs_on_kernel1_and_writes_back(monkeypatch):
    monkeypatch.setattr(solver.args, "pruning_factor", 0)
    dev = GpuDevice(0)
    try:
        eng = symref.Engine()

        def handler(st):
            try:
                return eng.step(st)
            except symref.Unsupported:
                eng.ended.append(("unsupported", st))
                return []
        laser = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy, execution_timeout=0,
                         escape_handler=handler)
        got, ends = Counter(), []
        laser.register_laser_hooks("transaction_end", lambda s, tx, ret, revert: got.update(
            [("txend", bool(revert), tuple(x.raw for x in s.world_state.constraints),
              s.environment.active_function_name)]))
        laser.register_laser_hooks("add_world_state", lambda s: (got.update(
            [("ws", tuple(x.raw for x in s.world_state.constraints))]), ends.append(s)))
        laser.work_list.append(bridge.pack_global_state(_symbolic_ref_state(), z))
        laser.exec()
        got += symcases._outcomes_of_restatement(eng)
        ref_eng = symref.Engine()
        ref_eng.run([bridge.pack_global_state(_symbolic_ref_state(), z)])
        want = symcases._outcomes_of_restatement(ref_eng)
        assert got == want
        assert laser.lane_steps > 100 and laser.forks >= 3 and ends
        # every kept world state writes back into a fresh reference object
        for s in ends:
            ref = _symbolic_ref_state()
            m0 = bridge.pack_global_state(ref, z)
            s.ref_n_constraints, s.ref_n_stores = m0.ref_n_constraints, m0.ref_n_stores
            bridge.unpack_global_state(s, ref, R.symbol_factory, R.smt, z)
            for w, rw in zip(s.mstate.stack, ref.mstate.stack):
                assert (rw.value if rw.value is not None else bridge.to_dag(rw.raw, z)) == \
                    (w.value if w.value is not None else w.raw)
            got_cons = [bridge.to_dag(c.raw, z) for c in ref.world_state.constraints]
            assert got_cons == [c.raw for c in s.world_state.constraints]
            chain = bridge.to_dag(ref.environment.active_account.storage._standard_storage.raw, z)
            assert chain is s.environment.active_account.storage.chain_raw()
    finally:
        dev.close()
