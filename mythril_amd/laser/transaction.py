"""Concrete message calls into the batched LASER core.

Mirrors transaction/concolic.py:75-151 (``execute_message_call`` and
``_setup_global_state_for_execution``) and the parts of
transaction/transaction_models.py:21-232 those use (tx ids, MessageCallTransaction,
initial_global_state with the value transfer).  Balances are concrete here: the
reference's ``UGE(balances[sender], value)`` conjunct is a constant for
concrete balances and is not recorded.
"""
from __future__ import annotations

from typing import List, Optional, Union

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
        self.call_data = bytes(call_data)
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
        value = concrete(self.call_value)
        if value:
            sender, receiver = concrete(env.sender), concrete(env.active_account.address)
            ws = gs.world_state
            if receiver in ws.accounts:
                ws.accounts[receiver].add_balance(value)
            if sender in ws.accounts:
                ws.accounts[sender].add_balance(-value)
        return gs

    def end(self, global_state: GlobalState, return_data=None, revert=False) -> None:
        self.return_data = return_data
        raise TransactionEndSignal(global_state, revert)

    def __str__(self):
        return "{} {} from {} to {:#42x}".format(type(self).__name__, self.id, self.caller,
                                                 concrete(self.callee_account.address))


def _setup_global_state_for_execution(laser_evm, transaction) -> None:
    global_state = transaction.initial_global_state()
    global_state.transaction_stack.append((transaction, None))
    global_state.world_state.transaction_sequence.append(transaction)
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
