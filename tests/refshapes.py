"""Test-only objects shaped like the reference's LASER state (mythril/laser/
ethereum/state/*.py and smt/*), exposing exactly the attributes
mythril_amd.bridge reads and writes: BitVec .value/.symbolic, Memory._memory
(keys are BitVecs) / _msize / extend / __getitem__ / __setitem__, Storage.
_standard_storage (K or Array) / printable_storage / __setitem__, Calldata
(_concrete_calldata for ConcreteCalldata; SymbolicCalldata has none), the
Environment words, MachineState, Account, WorldState, GlobalState with
transaction_stack.  The reference itself is not importable here (z3, eth_abi
and py-evm are absent), so these stand in for it."""


import fakez3 as _z


class BitVec:
    """value (None when symbolic) and, for a symbolic word, ``raw``: its z3
    term (the fake z3's), as the reference's BitVec.raw."""

    def __init__(self, value=None, size=256, name=None, raw=None):
        self.value, self._size, self.name = value, size, name
        if raw is None and value is None and name is not None:
            raw = _z.BitVec(name, size)
        self.raw = raw

    @property
    def symbolic(self):
        return self.value is None

    def size(self):
        return self._size

    def __hash__(self):
        return hash((self.value, self.name, id(self.raw) if self.value is None else 0))

    def __eq__(self, other):
        return isinstance(other, BitVec) and (self.value, self.name) == (other.value, other.name) and (
            self.value is not None or self.raw is other.raw)


class Bool:
    def __init__(self, raw):
        self.raw = raw
        self.value = None


class Smt:                                      # the mythril.laser.smt surface unpack uses
    @staticmethod
    def BitVec(raw):
        return BitVec(None, raw.sort().size(), raw=raw)

    Bool = Bool


smt = Smt()


def _raw(x, w=256):
    return _z.BitVecVal(x.value, w) if x.value is not None else x.raw


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


class K:                                       # array.py:73-86
    def __init__(self):
        self.raw = _z.K(256, _z.BitVecVal(0, 256))


class Array:                                   # array.py:56-70
    def __init__(self, name):
        self.raw = _z.Array(name, 256, 256)


class Storage:                                 # account.py:18-99
    def __init__(self, concrete=True, address=0):
        self._standard_storage = K() if concrete else Array(f"Storage{address}")
        self.printable_storage = {}
        self.keys_set = set()

    def __setitem__(self, key, value):
        self.printable_storage[key] = value
        self.keys_set.add(key)
        std = self._standard_storage
        std.raw = _z.Store(std.raw, _raw(key), _raw(value))


class Disassembly:
    def __init__(self, code_hex):
        self.bytecode = code_hex


class Account:
    def __init__(self, address, code_hex, concrete_storage=True, balance=0):
        self.address = BitVec(address)
        self.code = Disassembly(code_hex)
        self.storage = Storage(concrete_storage, address)
        self.nonce = 0
        self.contract_name = "Test"
        self._balance = BitVec(balance)

    def balance(self):
        return self._balance


class ConcreteCalldata:
    def __init__(self, data: bytes):
        self._concrete_calldata = list(data)


class SymbolicCalldata:                        # calldata.py:214-262 (tx_id)
    def __init__(self, tx_id="1"):
        self.tx_id = tx_id


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
