"""Concrete message calls and contract creations into the batched LASER core.

Mirrors transaction/concolic.py:23-151 (``execute_contract_creation``,
``execute_message_call`` and ``_setup_global_state_for_execution``) and the parts
of transaction/transaction_models.py:21-284 those use (tx ids,
MessageCallTransaction, ContractCreationTransaction, initial_global_state with the
value transfer, the creation ``end`` that installs the returned runtime code).
Balances live in the world state's symbolic ``Array("balance")`` as in the
reference: every transaction's initial state appends ``UGE(balances[sender],
value)`` and moves the value (transaction_models.py:127-148).

A creation transaction's calldata is the reference's ``SymbolicCalldata``
(concolic.py:57-70 passes ``call_data=None``): its lanes carry
MG_LANE_CREATION, so CALLDATALOAD/SIZE/COPY, CODESIZE and a CODECOPY from at or
past the end of the code (constructor arguments) escape to the host; an
argument-less constructor (CODECOPY of its own runtime code, RETURN) runs on the
device end to end.
"""
from __future__ import annotations

from typing import List, Optional, Union

from ..keccak import keccak256
from .disassembly import Disassembly
from .state import (Account, Environment, GlobalState, WorldState, concrete)


class TxIdManager:
    """transaction_models.py:21-36 (process-global counter)."""

    def __init__(self):
        self._next_transaction_id = 0

    def get_next_tx_id(self) -> str:
        self._next_transaction_id += 1
        return str(self._next_transaction_id)

    def restart_counter(self):
        self._next_transaction_id = 0

    def set_counter(self, tx_id):
        self._next_transaction_id = tx_id


tx_id_manager = TxIdManager()


class TransactionEndSignal(Exception):
    def __init__(self, global_state: GlobalState, revert: bool = False):
        self.global_state = global_state
        self.revert = revert


class MessageCallTransaction:
    """transaction_models.py:172-232 (concrete calldata and value)."""

    def __init__(self, world_state: WorldState, callee_account: Account = None, caller=None,
                 call_data: bytes = b"", identifier: Optional[str] = None, gas_price=0,
                 gas_limit=None, origin=None, code: Optional[Disassembly] = None, call_value=0,
                 static: bool = False, base_fee=0):
        self.world_state = world_state
        self.id = identifier or tx_id_manager.get_next_tx_id()
        self.gas_price = gas_price
        self.gas_limit = gas_limit
        self.origin = origin
        self.code = code
        self.caller = caller
        self.callee_account = callee_account
        # bytes, or a laser.symbolic.SymbolicCalldata for a symbolic transaction
        self.call_data = call_data if hasattr(call_data, "get_word_at") else bytes(call_data)
        self.call_value = call_value
        self.static = static
        self.base_fee = base_fee
        self.return_data: Optional[bytes] = None

    def initial_global_state(self) -> GlobalState:
        env = Environment(self.callee_account, self.caller, self.call_data, self.gas_price,
                          self.call_value, self.origin, self.base_fee,
                          code=self.code or self.callee_account.code, static=self.static)
        gs = GlobalState(self.world_state, env, None)
        gs.environment.active_function_name = "fallback"
        return _transfer_call_value(gs)

    def end(self, global_state: GlobalState, return_data=None, revert=False) -> None:
        self.return_data = return_data
        raise TransactionEndSignal(global_state, revert)

    def __str__(self):
        return "{} {} from {} to {:#42x}".format(type(self).__name__, self.id, self.caller,
                                                 concrete(self.callee_account.address))


def _transfer_call_value(gs: GlobalState) -> GlobalState:
    """transaction_models.py:127-148 (initial_global_state_from_environment):
    ``UGE(balances[sender], value)`` joins the path constraints, then the value
    moves from the sender's balance to the receiver's."""
    from ..smt.expr import UGE
    env, ws = gs.environment, gs.world_state
    value = env.callvalue
    ws.constraints.append(UGE(ws.balances[env.sender], value))
    ws.balances[env.active_account.address] = ws.balances[env.active_account.address] + value
    ws.balances[env.sender] = ws.balances[env.sender] - value
    return gs


# transaction/symbolic.py:28-40 Actors
ACTORS = {"CREATOR": 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,
          "ATTACKER": 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
          "SOMEGUY": 0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA}


def execute_symbolic_message_call(laser_evm, callee_address, gas_limit: int = 8_000_000,
                                  ids=None) -> None:
    """transaction/symbolic.py:105-150: one message call per open world state
    with symbolic calldata (``{id}_calldata``, ``{id}_calldatasize``), a
    symbolic sender/origin (``sender_{id}``), gas price and call value, plus
    the constraint that the sender is one of the ACTORS
    (symbolic.py:202-219); then ``laser_evm.exec()``.  The lanes run on the
    device as symbolic lanes (mythril_amd/laser/symbolic.py).  ``ids``: the
    transaction ids to use, one per open state (sharded runs: the states'
    global positions), instead of the counter's next ones."""
    from ..smt.expr import Or, symbol_factory
    from .symbolic import SymbolicCalldata
    open_states = laser_evm.open_states[:]
    del laser_evm.open_states[:]
    for k, ws in enumerate(open_states):
        acct = ws[callee_address]
        if getattr(acct, "deleted", False):
            continue
        txid = tx_id_manager.get_next_tx_id() if ids is None else ids[k]
        sender = symbol_factory.BitVecSym(f"sender_{txid}", 256)
        tx = MessageCallTransaction(
            world_state=ws, identifier=txid,
            gas_price=symbol_factory.BitVecSym(f"gas_price{txid}", 256), gas_limit=gas_limit,
            origin=sender, caller=sender, callee_account=acct, call_data=SymbolicCalldata(txid),
            call_value=symbol_factory.BitVecSym(f"call_value{txid}", 256))
        gs = tx.initial_global_state()
        gs.transaction_stack.append((tx, None))
        gs.world_state.constraints.append(
            Or(*[tx.caller == symbol_factory.BitVecVal(a, 256) for a in ACTORS.values()]))
        gs.world_state.transaction_sequence.append(tx)
        laser_evm.transaction_node(gs, tx)
        laser_evm.work_list.append(gs)
    laser_evm.exec()


def execute_symbolic_contract_creation(laser_evm, contract_initialization_code, contract_name=None,
                                       world_state=None, origin=ACTORS["CREATOR"], caller=ACTORS["CREATOR"]):
    """transaction/symbolic.py:154-200 (execute_contract_creation): one creation
    from `world_state` (a fresh one when None) with a symbolic gas price and
    call value and symbolic calldata (SymbolicCalldata(id): constructor
    arguments are read past the end of the code, instructions.py:979-1104);
    then ``laser_evm.exec(True)``.  Returns the new account.  The lanes run on
    the device as symbolic lanes: CALLDATA*, CODESIZE and CODECOPY past the
    end of the code included (k_sym_step)."""
    from ..smt.expr import symbol_factory
    from .symbolic import SymbolicCalldata
    world_state = world_state or WorldState()
    del laser_evm.open_states[:]
    txid = tx_id_manager.get_next_tx_id()
    code = contract_initialization_code
    tx = ContractCreationTransaction(
        world_state=world_state, identifier=txid,
        gas_price=symbol_factory.BitVecSym(f"gas_price{txid}", 256), gas_limit=8_000_000,
        origin=origin, code=code if isinstance(code, Disassembly) else Disassembly(code), caller=caller,
        contract_name=contract_name, call_data=SymbolicCalldata(txid),
        call_value=symbol_factory.BitVecSym(f"call_value{txid}", 256))
    # transaction/symbolic.py:202-219 (its _setup_global_state_for_execution
    # also pins the caller to the actors)
    from ..smt.expr import Or
    gs = tx.initial_global_state()
    gs.transaction_stack.append((tx, None))
    gs.world_state.constraints.append(
        Or(*[tx.caller == symbol_factory.BitVecVal(a, 256) for a in ACTORS.values()]))
    gs.world_state.transaction_sequence.append(tx)
    laser_evm.transaction_node(gs, tx)
    laser_evm.work_list.append(gs)
    new_account = tx.callee_account
    laser_evm.exec(True)
    return new_account


def _rlp_item(b: bytes) -> bytes:
    if len(b) == 1 and b[0] < 0x80:
        return b
    assert len(b) < 56
    return bytes([0x80 + len(b)]) + b


def _int_bytes(x: int) -> bytes:
    """rlp's big_endian_int sedes: minimal big-endian bytes, 0 -> b''."""
    return x.to_bytes((x.bit_length() + 7) // 8, "big") if x else b""


def generate_contract_address(creator: int, nonce: int) -> int:
    """py-evm ``eth._utils.address.generate_contract_address`` (used at
    world_state.py:237): keccak256(rlp([sender, nonce]))[12:].  The reference
    passes the creator as an int (its account key), which rlp encodes like the
    nonce: minimal big-endian bytes, so leading zero bytes of the address drop."""
    sender = _rlp_item(_int_bytes(creator))
    n = _rlp_item(_int_bytes(nonce))
    payload = sender + n
    return int.from_bytes(keccak256(bytes([0xC0 + len(payload)]) + payload)[12:], "big")


def create_account(world_state: WorldState, balance=0, address=None, concrete_storage=False,
                   creator=None, code=None, nonce=0) -> Account:
    """world_state.py:142-186: the creator's nonce picks the new address (and is
    bumped); a missing creator account is created first."""
    accounts = world_state.accounts
    if creator is not None:
        creator = concrete(creator)
    if creator in accounts:
        nonce = accounts[creator].nonce
    elif creator:
        create_account(world_state, address=creator)
    if address is None:
        if not creator:
            raise ValueError("a concrete creation needs a creator (the reference draws a random address)")
        address = generate_contract_address(creator, accounts[creator].nonce)
    if creator:
        accounts[creator].nonce += 1
    acct = Account(address, code=code, concrete_storage=concrete_storage, nonce=nonce,
                   balances=world_state.balances)
    acct.set_balance(balance)
    world_state.put_account(acct)
    return acct


class ContractCreationTransaction(MessageCallTransaction):
    """transaction_models.py:206-284: a fresh account (concrete storage) runs the
    creation code; ``end`` with non-empty return data installs it as the
    account's code and returns the address, otherwise the world state is not
    kept (svm.py:459-466)."""

    def __init__(self, world_state: WorldState, caller=None, call_data=None, identifier=None,
                 gas_price=0, gas_limit=None, origin=None, code: Optional[Disassembly] = None,
                 call_value=0, contract_name=None, contract_address=None, base_fee=0):
        contract_address = contract_address if isinstance(contract_address, int) else None
        callee_account = create_account(world_state, 0, concrete_storage=True, creator=caller,
                                        address=contract_address)
        callee_account.contract_name = contract_name or callee_account.contract_name
        # a SymbolicCalldata object (transaction/symbolic.py's creation) is the
        # environment's calldata; None (concolic creation) keeps an empty concrete
        # calldata whose CALLDATA* / CODESIZE escape to the host's handler
        symcd = call_data is not None and hasattr(call_data, "get_word_at")
        super().__init__(world_state, callee_account, caller, call_data if symcd else b"", identifier,
                         gas_price, gas_limit, origin, code, call_value, False, base_fee)
        self.symbolic_calldata = call_data is None or symcd

    def initial_global_state(self) -> GlobalState:
        gs = super().initial_global_state()
        gs.environment.active_function_name = "constructor"
        return gs

    def end(self, global_state: GlobalState, return_data=None, revert=False) -> None:
        if not return_data:
            self.return_data = None
            raise TransactionEndSignal(global_state, revert)
        install_runtime_code(self, global_state, return_data)
        raise TransactionEndSignal(global_state, revert)


def install_runtime_code(tx: ContractCreationTransaction, global_state: GlobalState,
                         return_data: bytes) -> None:
    """transaction_models.py:277-283: assign_bytecode(return data) on the active
    account; the transaction's return data becomes the account's address."""
    account = global_state.environment.active_account
    account.code = Disassembly(bytes(return_data))
    if concrete(account.address) in global_state.world_state.accounts:
        global_state.world_state.accounts[concrete(account.address)].code = account.code
    tx.return_data = hex(concrete(account.address))
    assert account.code.instruction_list != []


def _setup_global_state_for_execution(laser_evm, transaction) -> None:
    global_state = transaction.initial_global_state()
    global_state.transaction_stack.append((transaction, None))
    global_state.world_state.transaction_sequence.append(transaction)
    laser_evm.transaction_node(global_state, transaction)
    laser_evm.work_list.append(global_state)


def execute_message_call(laser_evm, callee_address, caller_address, origin_address, data, gas_limit,
                         gas_price, value, code=None, track_gas=False
                         ) -> Union[None, List[GlobalState]]:
    """concolic.execute_message_call: one MessageCallTransaction per open world
    state, then ``laser_evm.exec(track_gas=track_gas)``."""
    open_states: List[WorldState] = laser_evm.open_states[:]
    del laser_evm.open_states[:]
    for open_world_state in open_states:
        next_transaction_id = tx_id_manager.get_next_tx_id()
        code = code or open_world_state[callee_address].code.bytecode
        transaction = MessageCallTransaction(
            world_state=open_world_state,
            identifier=next_transaction_id,
            gas_price=gas_price,
            gas_limit=gas_limit,
            origin=origin_address,
            code=Disassembly(code),
            caller=caller_address,
            callee_account=open_world_state[callee_address],
            call_data=data,
            call_value=value,
        )
        _setup_global_state_for_execution(laser_evm, transaction)
    return laser_evm.exec(track_gas=track_gas)


def execute_contract_creation(laser_evm, callee_address, caller_address, origin_address, data,
                              gas_limit, gas_price, value, code=None, track_gas=False,
                              contract_name=None) -> Union[None, List[GlobalState]]:
    """concolic.execute_contract_creation (concolic.py:23-72): one
    ContractCreationTransaction per open world state running ``data`` as the
    creation code (symbolic calldata), then ``laser_evm.exec(True, track_gas)``."""
    open_states: List[WorldState] = laser_evm.open_states[:]
    del laser_evm.open_states[:]
    for open_world_state in open_states:
        next_transaction_id = tx_id_manager.get_next_tx_id()
        transaction = ContractCreationTransaction(
            world_state=open_world_state,
            identifier=next_transaction_id,
            gas_price=gas_price,
            gas_limit=gas_limit,
            origin=origin_address,
            code=Disassembly(data),
            caller=caller_address,
            contract_name=contract_name,
            call_data=None,
            call_value=value,
        )
        _setup_global_state_for_execution(laser_evm, transaction)
    return laser_evm.exec(True, track_gas=track_gas)
