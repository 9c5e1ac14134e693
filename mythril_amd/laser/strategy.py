"""Search strategies (strategy/__init__.py:7-33, strategy/basic.py:10-49).

For the batched core a strategy decides two things: which states of the work
list are dropped before they run (``max_depth``, as ``BasicSearchStrategy.__next__``),
and the ORDER in which per-path events — hooks, halts, open world states,
final states — are delivered to the host, which is the order the reference's
one-state-at-a-time loop would produce:

* BFS pops the oldest state, so concrete paths advance round-robin: the k-th
  instruction of every path runs before any path's (k+1)-th.  Events are
  delivered by (instruction round, work-list position).
* DFS pops the newest state and runs it to its end before the next: events are
  delivered by (reverse work-list position, instruction round).
"""
from __future__ import annotations

from abc import ABC
from typing import List


class BasicSearchStrategy(ABC):
    #: "bfs" or "dfs": event delivery order of LaserEVM.exec
    order = "bfs"

    def __init__(self, work_list, max_depth, **kwargs):
        self.work_list = work_list
        self.max_depth = max_depth

    def run_check(self) -> bool:
        return True

    def drain(self) -> List:
        """Remove and return every runnable state of the work list (states at or
        beyond max_depth are skipped, as __next__ skips them)."""
        states = [s for s in self.work_list if s.mstate.depth < self.max_depth]
        del self.work_list[:]
        return states


class DepthFirstSearchStrategy(BasicSearchStrategy):
    order = "dfs"


class BreadthFirstSearchStrategy(BasicSearchStrategy):
    order = "bfs"


class JumpdestCountAnnotation:
    """bounded_loops.py:14-26: the addresses of the instructions the path was
    popped at.  While the path runs on kernel 1 the trace lives in the lane's
    device buffer; it is written back here whenever the state is materialised."""

    def __init__(self):
        self._reached_count = {}
        self.trace: List[int] = []

    def __copy__(self):
        out = JumpdestCountAnnotation()
        out._reached_count = dict(self._reached_count)
        out.trace = list(self.trace)
        return out


class BoundedLoopsStrategy(BasicSearchStrategy):
    """bounded_loops.py:29-145 as a strategy extension
    (``laser.extend_strategy(BoundedLoopsStrategy, loop_bound=3)``).  The trace
    append and the loop count at every JUMPDEST run on the device
    (mg_set_loop_bound); a dropped path stops with MG_LOOP_BOUND and is never
    returned to the execution loop, as the reference's ``continue`` skips it."""

    def __init__(self, super_strategy: BasicSearchStrategy, **kwargs):
        self.super_strategy = super_strategy
        self.bound = kwargs["loop_bound"]
        self.order = getattr(super_strategy, "order", "bfs")
        BasicSearchStrategy.__init__(self, super_strategy.work_list, super_strategy.max_depth,
                                     **kwargs)

    def drain(self) -> List:
        return self.super_strategy.drain()

    @staticmethod
    def get_loop_count(trace: List[int]) -> int:
        """get_loop_count of a host-held trace (the device computes the same
        count at every JUMPDEST).  Segments are compared by their OR-of-shifted
        hash one byte at a time: byte k is lo8(S[k]) | hi8(S[k-1]) for 16-bit
        addresses (EVM code is < 64 KiB)."""
        n = len(trace)
        last2 = (trace[-2], trace[-1]) if n >= 2 else None
        start = next((i for i in range(n - 3, 0, -1) if (trace[i], trace[i + 1]) == last2), None)
        if start is None:
            return 0
        base, size = start + 1, n - start - 2

        def hash_bytes(at):
            seg = trace[at: at + size] + [0]
            return [(seg[k] & 0xFF) | ((seg[k - 1] >> 8) if k else 0) for k in range(size + 1)]

        key = hash_bytes(base)
        count, j = 2, base - size
        while j >= 0 and hash_bytes(j) == key:
            count += 1
            j -= size
        return count


class DelayConstraintStrategy(BasicSearchStrategy):
    """constraint_strategy.py:19-47: a state whose path constraints no cached
    model satisfies (``check_quick_sat`` on the strategy's OWN ModelCache —
    kernel 2) is parked; parked states run only once the work list is empty,
    each after ``Constraints.get_model`` (global cache, then the SMT backend)
    finds it a model, which then joins the strategy's cache.  States pop in
    work-list order (``pop(0)``).  Batched form: ``drain`` returns every
    runnable state at once in that order, or the first parked state that gets
    a model; the quick-sat checks of one drain go to the device in ONE
    kernel-2 launch (``check_quick_sat_many`` replays them in order)."""

    order = "bfs"

    def __init__(self, work_list, max_depth, **kwargs):
        super().__init__(work_list, max_depth)
        from ..smt.solver import ModelCache
        self.model_cache = ModelCache(device=kwargs.get("device"))
        self.pending_worklist: List = []
        # a parked state whose query neither a candidate model nor an SMT backend
        # can decide (SolverBackendMissing): "raise", or "keep" it running without
        # a model to cache (prefilter-only runs, as LaserEVM.unknown_forks)
        self.unknown = "raise"
        self.unknown_kept = 0

    def drain(self) -> List:
        from ..smt.expr import And
        from ..smt.solver import Constraints
        states = [s for s in self.work_list if s.mstate.depth < self.max_depth]
        del self.work_list[:]
        if states:
            queries = [And(*s.world_state.constraints).raw for s in states]
            verdicts = self.model_cache.check_quick_sat_many(queries)
            run = []
            for s, v in zip(states, verdicts):
                (run if v is not False else self.pending_worklist).append(s)
            if run:
                return run
        from ..smt.solver import SolverBackendMissing
        while self.pending_worklist:
            s = self.pending_worklist.pop(0)
            try:
                model = Constraints(s.world_state.constraints).get_model()
            except SolverBackendMissing:
                if self.unknown != "keep":
                    raise
                self.unknown_kept += 1
                return [s]
            if model is not None:
                self.model_cache.put(model, 1)
                return [s]
        return []
