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
