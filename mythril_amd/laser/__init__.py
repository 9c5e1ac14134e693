"""Host side of the batched LASER core: the reference's LaserEVM / GlobalState /
hook / plugin surface (mythril/laser/ethereum), stepping paths on kernel 1."""
from .disassembly import Disassembly, disassemble
from .plugins import InstructionCoveragePlugin, LaserPlugin
from .signals import PluginSkipState, PluginSkipWorldState
from .state import (Account, Environment, GlobalState, MachineStack, MachineState, Memory,
                    Storage, WorldState)
from .strategy import (BoundedLoopsStrategy, BreadthFirstSearchStrategy, DepthFirstSearchStrategy,
                       JumpdestCountAnnotation)
from .svm import LaserEVM
from .transaction import MessageCallTransaction, execute_message_call, tx_id_manager

__all__ = ["Account", "BoundedLoopsStrategy", "BreadthFirstSearchStrategy",
           "JumpdestCountAnnotation", "DepthFirstSearchStrategy", "Disassembly",
           "Environment", "GlobalState", "InstructionCoveragePlugin", "LaserEVM", "LaserPlugin",
           "MachineStack", "MachineState", "Memory", "MessageCallTransaction",
           "PluginSkipState", "PluginSkipWorldState", "Storage", "WorldState", "disassemble",
           "execute_message_call", "tx_id_manager"]
