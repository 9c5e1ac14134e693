"""The statespace graph (laser/ethereum/cfg.py): nodes are the straight-line
pieces of a path between JUMP / JUMPI / call-return boundaries, edges the
transfers between them.  LaserEVM builds it when ``requires_statespace`` is set
(svm.py:549-637), stepping every state one instruction at a time so that each
node lists the states of its instructions as the reference's does."""
from __future__ import annotations

from enum import Enum, IntFlag
from typing import Dict, List


class JumpType(Enum):
    """cfg.py:11-18."""
    CONDITIONAL = 1
    UNCONDITIONAL = 2
    CALL = 3
    RETURN = 4
    Transaction = 5


class NodeFlags(IntFlag):
    """cfg.py:21-29 (the reference's `flags.Flags`; an empty value is falsy)."""
    FUNC_ENTRY = 1
    CALL_RETURN = 2


class Node:
    """cfg.py:32-82: one node of the graph; ``states`` holds the state at each
    instruction of the node, ``uid`` is the object's hash as in the reference."""

    def __init__(self, contract_name: str, start_addr=0, constraints=None,
                 function_name="unknown") -> None:
        from ..smt.solver import Constraints
        self.contract_name = contract_name
        self.start_addr = start_addr
        self.states: List = []
        self.constraints = constraints if constraints else Constraints()
        self.function_name = function_name
        self.flags = NodeFlags(0)
        self.uid = hash(self)

    def get_cfg_dict(self) -> Dict:
        code = ""
        for state in self.states:
            instruction = state.get_current_instruction()
            code += str(instruction["address"]) + " " + instruction["opcode"]
            if instruction["opcode"].startswith("PUSH"):
                code += " " + "".join(str(instruction["argument"]))
            code += "\\n"
        return dict(contract_name=self.contract_name, start_addr=self.start_addr,
                    function_name=self.function_name, code=code)


class Edge:
    """cfg.py:85-120."""

    def __init__(self, node_from: int, node_to: int, edge_type=JumpType.UNCONDITIONAL,
                 condition=None) -> None:
        self.node_from = node_from
        self.node_to = node_to
        self.type = edge_type
        self.condition = condition

    def __str__(self) -> str:
        return str(self.as_dict)

    @property
    def as_dict(self) -> Dict[str, int]:
        return {"from": self.node_from, "to": self.node_to}
