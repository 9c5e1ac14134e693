"""LASER plugins whose effect the device reproduces (SURVEY §8(b) batch-safe hooks).

``InstructionCoveragePlugin`` mirrors plugin/plugins/coverage/coverage_plugin.py:21-118:
same ``coverage`` table ({bytecode: (n_instructions, [covered])}), same
``start_sym_trans``/``stop_sym_trans``/``stop_sym_exec`` reporting, but the
per-instruction marks come from kernel 1's coverage bytes instead of an
``execute_state`` hook (which would stop every lane at every instruction).
Across GPUs the bytes are OR-all-gathered over RCCL (bench.py, §8(e)).
"""
from __future__ import annotations

import logging

log = logging.getLogger(__name__)


class LaserPlugin:
    """plugin/interface.py: ``initialize(symbolic_vm)``."""

    def initialize(self, symbolic_vm) -> None:
        raise NotImplementedError


class InstructionCoveragePlugin(LaserPlugin):
    def __init__(self):
        self.coverage = {}
        self.initial_coverage = 0
        self.tx_id = 0
        self._vm = None

    def initialize(self, symbolic_vm) -> None:
        self.coverage = {}
        self.initial_coverage = 0
        self.tx_id = 0
        self._vm = symbolic_vm
        symbolic_vm.record_coverage = True

        @symbolic_vm.laser_hook("stop_exec")
        def stop_exec_hook():
            self.coverage = symbolic_vm.coverage()

        @symbolic_vm.laser_hook("stop_sym_exec")
        def stop_sym_exec_hook():
            self.coverage = symbolic_vm.coverage()
            for code, (n, bits) in self.coverage.items():
                pct = 0 if n == 0 else sum(bits) / float(n) * 100
                log.info("Achieved {:.2f}% coverage for code: {}".format(pct, code))

        @symbolic_vm.laser_hook("start_sym_trans")
        def execute_start_sym_trans_hook():
            self.initial_coverage = self._get_covered_instructions()

        @symbolic_vm.laser_hook("stop_sym_trans")
        def execute_stop_sym_trans_hook():
            self.coverage = symbolic_vm.coverage()
            end_coverage = self._get_covered_instructions()
            log.info("Number of new instructions covered in tx %d: %d"
                     % (self.tx_id, end_coverage - self.initial_coverage))
            self.tx_id += 1

    def _get_covered_instructions(self) -> int:
        return sum(sum(cv[1]) for cv in self.coverage.values())

    def is_instruction_covered(self, bytecode, index) -> bool:
        if bytecode not in self.coverage:
            return False
        try:
            return self.coverage[bytecode][1][index]
        except IndexError:
            return False
