"""KeccakFunctionManager (laser/ethereum/function_managers/keccak_function_manager.py:
24-179) on the device-evaluable expression layer.

Symbolic SHA3 inputs become applications of ``keccak256_<bits>`` with an inverse
``keccak256_<bits>-1``; concrete inputs are hashed (Keccak-256) and recorded.
``create_conditions`` builds the conjunct every ``get_all_constraints`` appends:
for each symbolic input, inverse(f(x)) == x and f(x) in its size's interval with
f(x) % 64 == 0, or equal to one of the concrete hashes of the same size; for
each concrete input, f(c) == h and inverse(f(c)) == c.  Intervals are assigned
per input size in first-use order (TOTAL_PARTS, PART, INTERVAL_DIFFERENCE as
the reference).  Kernel 2 evaluates these conjuncts through its table op
(keys up to 512 bits: mapping slots), see lower.py.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from ..keccak import keccak256
from .expr import And, BitVec, Bool, Function, Or, ULE, ULT, URem, symbol_factory

TOTAL_PARTS = 10 ** 40
PART = (2 ** 256 - 1) // TOTAL_PARTS
INTERVAL_DIFFERENCE = 10 ** 30


class KeccakFunctionManager:
    hash_matcher = "fffffff"

    def __init__(self):
        # set once: reset() keeps the counter (keccak_function_manager.py:38-54), so
        # sizes first seen after a reset get fresh, lower intervals
        self._index_counter = TOTAL_PARTS - 34534
        self.reset()

    def reset(self):
        try:                                  # the search's term-dependency memo holds terms
            from .search import clear_deps
            clear_deps()
        except ImportError:
            pass
        self.store_function: Dict[int, Tuple[Function, Function]] = {}
        self.interval_hook_for_size: Dict[int, int] = {}
        self.hash_result_store: Dict[int, List[BitVec]] = {}
        self.quick_inverse: Dict[BitVec, BitVec] = {}
        self.concrete_hashes: Dict[BitVec, BitVec] = {}
        self.symbolic_inputs: Dict[int, List[BitVec]] = {}

    @staticmethod
    def find_concrete_keccak(data: BitVec) -> BitVec:
        return symbol_factory.BitVecVal(
            int.from_bytes(keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256)

    def get_function(self, length: int) -> Tuple[Function, Function]:
        try:
            func, inverse = self.store_function[length]
        except KeyError:
            func = Function("keccak256_{}".format(length), [length], 256)
            inverse = Function("keccak256_{}-1".format(length), [256], length)
            self.store_function[length] = (func, inverse)
            self.hash_result_store[length] = []
        return func, inverse

    @staticmethod
    def get_empty_keccak_hash() -> BitVec:
        return symbol_factory.BitVecVal(
            89477152217924674838424037953991966239322087453347756267410168184682657981552, 256)

    def create_keccak(self, data: BitVec) -> BitVec:
        length = data.size()
        func, _ = self.get_function(length)
        if data.symbolic is False:
            concrete_hash = self.find_concrete_keccak(data)
            self.concrete_hashes[data] = concrete_hash
            return concrete_hash
        self.symbolic_inputs.setdefault(length, []).append(data)
        self.hash_result_store[length].append(func(data))
        return func(data)

    def register_concrete(self, data: bytes, hash_value: int) -> BitVec:
        """create_keccak for a concrete input whose hash the device already
        computed (an MG_REC_KECCAK record of kernel 1): the same get_function
        side effect and concrete_hashes entry, keyed by the 8*len-bit input."""
        bv = symbol_factory.BitVecVal(int.from_bytes(data, "big"), 8 * len(data))
        self.get_function(bv.size())
        h = symbol_factory.BitVecVal(hash_value, 256)
        self.concrete_hashes[bv] = h
        return h

    def assign_intervals(self) -> None:
        """The interval hooks create_conditions assigns (sizes in first-use
        order), without building the conditions (search.complete needs only
        the intervals)."""
        for length in self.symbolic_inputs:
            if length not in self.interval_hook_for_size:
                self.interval_hook_for_size[length] = self._index_counter
                self._index_counter -= INTERVAL_DIFFERENCE

    def create_conditions(self) -> Bool:
        condition = symbol_factory.Bool(True)
        for inputs_list in self.symbolic_inputs.values():
            for symbolic_input in inputs_list:
                condition = And(condition, self._create_condition(func_input=symbolic_input))
        for concrete_input, concrete_hash in self.concrete_hashes.items():
            func, inverse = self.get_function(concrete_input.size())
            condition = And(condition, func(concrete_input) == concrete_hash,
                            inverse(func(concrete_input)) == concrete_input)
        return condition

    def _create_condition(self, func_input: BitVec) -> Bool:
        length = func_input.size()
        func, inv = self.get_function(length)
        try:
            index = self.interval_hook_for_size[length]
        except KeyError:
            self.interval_hook_for_size[length] = self._index_counter
            index = self._index_counter
            self._index_counter -= INTERVAL_DIFFERENCE
        lower_bound = index * PART
        upper_bound = lower_bound + PART
        cond = And(
            inv(func(func_input)) == func_input,
            ULE(symbol_factory.BitVecVal(lower_bound, 256), func(func_input)),
            ULT(func(func_input), symbol_factory.BitVecVal(upper_bound, 256)),
            URem(func(func_input), symbol_factory.BitVecVal(64, 256)) == 0,
        )
        concrete_cond = symbol_factory.Bool(False)
        for key, keccak in self.concrete_hashes.items():
            if key.size() == func_input.size():
                hash_eq = And(func(func_input) == keccak, key == func_input)
                concrete_cond = Or(concrete_cond, hash_eq)
        return And(inv(func(func_input)) == func_input, Or(cond, concrete_cond))

    def get_concrete_hash_data(self, model) -> Dict[int, List[Optional[int]]]:
        """Concrete hash values per input size under `model` (solver.Model /
        ModelRef): model.eval of every symbolic hash application, without model
        completion; the ones that stay symbolic are skipped."""
        out: Dict[int, List[Optional[int]]] = {}
        for size, vals in self.hash_result_store.items():
            out[size] = []
            for val in vals:
                ev = model.eval(val.raw)
                if ev is not None and ev.op == "const":
                    out[size].append(ev.param)
        return out


keccak_function_manager = KeccakFunctionManager()
