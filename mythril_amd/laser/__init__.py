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
from .cfg import Edge, JumpType, Node, NodeFlags
from .transaction import (ContractCreationTransaction, MessageCallTransaction,
                          execute_contract_creation, execute_message_call, execute_symbolic_message_call,
                          execute_symbolic_contract_creation,
                          generate_contract_address, tx_id_manager)
from .symbolic import SymbolicCalldata

__all__ = ["Account", "BoundedLoopsStrategy", "BreadthFirstSearchStrategy",
           "ContractCreationTransaction", "execute_contract_creation", "generate_contract_address",
           "JumpdestCountAnnotation", "DepthFirstSearchStrategy", "Disassembly",
           "Environment", "GlobalState", "InstructionCoveragePlugin", "LaserEVM", "LaserPlugin",
           "MachineStack", "MachineState", "Memory", "MessageCallTransaction",
           "PluginSkipState", "PluginSkipWorldState", "Storage", "WorldState", "disassemble",
           "execute_message_call", "execute_symbolic_message_call", "execute_symbolic_contract_creation", "SymbolicCalldata", "tx_id_manager"]
