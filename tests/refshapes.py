"""Test-only objects shaped like the reference's LASER state (mythril/laser/
ethereum/state/*.py and smt/*), exposing exactly the attributes
mythril_amd.bridge reads and writes: BitVec .value/.symbolic, Memory._memory
(keys are BitVecs) / _msize / extend / __getitem__ / __setitem__, Storage.
_standard_storage (K or Array) / printable_storage / __setitem__, Calldata
(_concrete_calldata for ConcreteCalldata; SymbolicCalldata has none), the
Environment words, MachineState, Account, WorldState, GlobalState with
transaction_stack.  The reference itself is not importable here (z3, eth_abi
and py-evm are absent), so these stand in for it."""


class BitVec:
    def __init__(self, value=None, size=256, name=None):
        self.value, self._size, self.name = value, size, name

    @property
    def symbolic(self):
        return self.value is None

    def size(self):
        return self._size

    def __hash__(self):
        return hash((self.value, self.name))

    def __eq__(self, other):
        return isinstance(other, BitVec) and (self.value, self.name) == (other.value, other.name)


class SymbolFactory:
    @staticmethod
    def BitVecVal(v, size):
        return BitVec(v % (1 << size), size)

    @staticmethod
    def BitVecSym(name, size):
        return BitVec(None, size, name)


symbol_factory = SymbolFactory()


class Memory:                                   # memory.py:28-208
    def __init__(self):
        self._msize = 0
        self._memory = {}

    def __len__(self):
        return self._msize

    def extend(self, size):
        self._msize += size

    def __getitem__(self, item):
        return self._memory.get(BitVec(item), 0)

    def __setitem__(self, key, value):
        if key >= len(self):
            return
        self._memory[BitVec(key)] = value


class K:                                       # array.py:73-86 (marker)
    pass


class Array:
    pass


class Storage:                                 # account.py:18-99
    def __init__(self, concrete=True):
        self._standard_storage = K() if concrete else Array()
        self.printable_storage = {}
        self.keys_set = set()

    def __setitem__(self, key, value):
        self.printable_storage[key] = value
        self.keys_set.add(key)


class Disassembly:
    def __init__(self, code_hex):
        self.bytecode = code_hex


class Account:
    def __init__(self, address, code_hex, concrete_storage=True, balance=0):
        self.address = BitVec(address)
        self.code = Disassembly(code_hex)
        self.storage = Storage(concrete_storage)
        self.nonce = 0
        self.contract_name = "Test"
        self._balance = BitVec(balance)

    def balance(self):
        return self._balance


class ConcreteCalldata:
    def __init__(self, data: bytes):
        self._concrete_calldata = list(data)


class SymbolicCalldata:
    pass


class Environment:
    def __init__(self, account, sender, calldata, gasprice, callvalue, origin):
        self.active_account = account
        self.code = account.code
        self.sender, self.calldata, self.gasprice = BitVec(sender), calldata, gasprice
        self.callvalue, self.origin = BitVec(callvalue), BitVec(origin)
        self.static = False


class MachineState:
    def __init__(self, gas_limit=10 ** 9):
        self.pc = 0
        self.stack = []
        self.memory = Memory()
        self.gas_limit = gas_limit
        self.min_gas_used = self.max_gas_used = 0
        self.depth = 0


class MessageCallTransaction:
    def __init__(self, gas_limit):
        self.gas_limit = gas_limit
        self.id = "1"


class WorldState:
    def __init__(self):
        self.transaction_sequence = []
        self.constraints = []


class GlobalState:
    def __init__(self, world_state, environment, mstate, tx):
        self.world_state, self.environment, self.mstate = world_state, environment, mstate
        self.transaction_stack = [(tx, None)]
        self.annotations = []

    @property
    def current_transaction(self):
        return self.transaction_stack[-1][0]
