"""ExponentFunctionManager (laser/ethereum/function_managers/exponent_function_manager.py:
10-63) on the device-evaluable expression layer.

EXP of two concrete operands yields the concrete power and the constraint
``result == Power(base, exponent)``, which instructions.py:624-638 appends to
the path's constraints; kernel 1 logs it as an MG_REC_EXP record and the host
replays it through ``create_condition`` when it materialises the lane.
Symbolic operands yield ``Power(base, exponent)`` with ``Power(...) > 0`` (signed,
as the reference's BitVec ``>``), the 256**i table for i < 32 and, for base 256,
periodicity of the exponent mod 32.
"""
from __future__ import annotations

from typing import Tuple

from .expr import And, BitVec, Bool, Function, URem, symbol_factory


class ExponentFunctionManager:
    def __init__(self):
        self.reset()
        power = Function("Power", [256, 256], 256)
        n256 = symbol_factory.BitVecVal(256, 256)
        self.concrete_constraints = And(*[
            power(n256, symbol_factory.BitVecVal(i, 256)) == symbol_factory.BitVecVal(256 ** i, 256)
            for i in range(0, 32)])

    def reset(self) -> None:
        """Forget the points registered by earlier runs (host bookkeeping only:
        the reference's manager keeps no per-run state, so this changes no
        constraint)."""
        # concrete (base, exponent) -> power of every EXP registered so far (what
        # a model must interpret Power as; laser/witness.py completes seeds with it)
        self.concrete_points = {(256, i): 256 ** i for i in range(32)}
        # (base, exponent) of every EXP with a symbolic operand (host bookkeeping:
        # a candidate model interprets Power at their values, laser/witness.py)
        self.symbolic_points = []

    def create_condition(self, base: BitVec, exponent: BitVec) -> Tuple[BitVec, Bool]:
        power = Function("Power", [256, 256], 256)
        exponentiation = power(base, exponent)
        if exponent.symbolic is False and base.symbolic is False:
            const = symbol_factory.BitVecVal(pow(base.value, exponent.value, 2 ** 256), 256,
                                             annotations=base.annotations.union(exponent.annotations))
            self.concrete_points[(base.value, exponent.value)] = const.value
            return const, const == exponentiation
        self.symbolic_points.append((base, exponent))
        constraint = And(exponentiation > 0, self.concrete_constraints)
        if base.value == 256:
            constraint = And(constraint,
                             power(base, URem(exponent, symbol_factory.BitVecVal(32, 256)))
                             == power(base, exponent))
        return exponentiation, constraint


exponent_function_manager = ExponentFunctionManager()
