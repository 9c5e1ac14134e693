"""Shared harness of the symbolic-lane tests (CPU with the oracle device,
MI355X with kernel 1): deploy a reference test contract concretely, run one
symbolic message call (transaction/symbolic.py:105-150) through the batched
LaserEVM, and the same call through the CPU restatement (tests/symref.py);
both sides report every path's outcome with its constraint sequence.

The fork filter is off on both sides (args.pruning_factor = 0): no SMT solver
exists here to prove a branch infeasible, so every fork is kept, as the
reference keeps them when the filter does not run (svm.py:319-326)."""
from __future__ import annotations

from collections import Counter

import symref
from mythril_amd import workloads
from mythril_amd.laser import (Account, BreadthFirstSearchStrategy, Disassembly, LaserEVM, MessageCallTransaction,
                               SymbolicCalldata, WorldState, execute_contract_creation,
                               execute_symbolic_message_call, generate_contract_address)
from mythril_amd.laser.transaction import ACTORS, tx_id_manager
from mythril_amd.smt import solver
from mythril_amd.smt.expr import Or, symbol_factory

CREATOR = ACTORS["CREATOR"]
# contract -> (creation code suffix: constructor arguments, call value of the creation)
CONTRACTS = {
    "flag_array.sol.o": (b"", 10 ** 17),                              # require(msg.value == 0.1 ether)
    "symbolic_exec_bytecode.sol.o": ((10).to_bytes(32, "big"), 0),  # _log2Size = 10
}


# runtime bytecode analysed as `myth analyze -f <code>` does without on-chain data:
# an account at a fixed address with the code and symbolic storage
# (analysis/symbolic.py:183-193: concrete_storage=False, Array("Storage{address}"))
RUNTIME = ("overflow.sol.o", "exceptions.sol.o", "environments.sol.o", "symkey_sha3", "selfbalance_ret", "balance_of", "symjump", "symlen_sha3", "gas_sym", "block_env", "log_sym", "memjump")

# synthetic runtime code: memory at a symbolic offset x = calldata[4:36] feeding
# SHA3 (sha3_ at a symbolic offset, instructions.py:1014-1051) and symbolic
# storage:  MSTORE(x, CALLER); h = SHA3(x, 64); if !storage[h]: storage[h] = 1;
# y = calldata[36:68]; if y: MSTORE8(x, y); if MLOAD(x): storage[0] = SHA3(x, 33)
SYNTH = {"symkey_sha3": "600435338152604081208054601357600181555b6024358015601f578083535b"
                        "825180602757005b6021842060005500",
         # b = SELFBALANCE; if b == 0: RETURN(0, b); x = calldata[0:32];
         # if b < x: REVERT(0, x); if x & 1: RETURN(x, 32); REVERT(x, 4) -- halts of a
         # symbolic length or offset (instructions.py:1858-1934)
         "selfbalance_ret": "478015602457600035808210601f5780600116601a57600481fd5b602081f35b806000fd5b806000f3",
         # BALANCE (instructions.py:907-931) of the contract's own address, of calldata[0:32],
         # of CALLER and of an unknown concrete address, each feeding a JUMPI
         "balance_of": "303160003531818111600d57005b333115601557005b61123431601e57005b00",
         # symbolic jump targets: JUMPI(x, x) falls through (instructions.py:1572-1579),
         # JUMP(x) raises InvalidJumpDestination (:1529-1532)
         "symjump": "600035806001166019578080576001600055602035602357005b801560215780565b005b00",
         # SHA3 of a symbolic length over symbolic memory: length 64 and `n == 64` on the path
         # (instructions.py:1023-1028)
         "symlen_sha3": "600035806000526020356000205460165780602857005b6040356010206000558015602657005b005b00",
         # GAS: the transaction's fresh "gas" variable (instructions.py:1700-1709) in JUMPI conditions
         "gas_sym": "5a600035106010575a600116601957005b5a15601757005b005b00",
         # NUMBER, TIMESTAMP, CHAINID, COINBASE, DIFFICULTY in JUMPI conditions (instructions.py:958-965,
         # 1386-1425)
         "block_env": "434210600e5746600114601657005b414411601857005b005b00",
         # LOG1 / LOG2 / LOG0 with symbolic topics, offset and length (log_, instructions.py:1710-1723)
         "log_sym": "6000353360006000a1808060206000a280600116601f5780600216602b57005b8015602657005b8080a0005b00",
         # a jump target read back from memory at a symbolic offset: MSTORE(x, 15),
         # JUMP(MLOAD(x)) with x = calldata[0:32] -- the MLOADK node decodes to the concrete 15
         # (get_word_at over the byte map), so the reference jumps; the device must hand the
         # jump to the host instead of raising InvalidJumpDestination
         # (then two calldata-bit branches, for paths past the jump)
         "memjump": "600035600f81525156" + "00" * 6 + "5b602035806001166021576002166028570"
                    "05b6001600055005b600260015500"}


# the other reference codes (tests/testdata/inputs/*.sol.o), deployed as RUNTIME codes
FIELD = [n for n in sorted(workloads.bytecode_names()) if n not in CONTRACTS and n not in RUNTIME]
ALL_CASES = sorted(CONTRACTS) + list(RUNTIME) + FIELD


def deploy(device, name):
    """Concolic creation (concolic.py:23-72) of a reference test contract (a
    RUNTIME code: the account holding it, with symbolic storage); returns (the
    open world state, the account's address)."""
    if name in RUNTIME or name not in CONTRACTS:
        ws = WorldState()
        ws.put_account(Account(CREATOR, balances=None))
        code = bytes.fromhex(SYNTH[name]) if name in SYNTH else workloads.bytecode(name)
        acct = Account(workloads.CONTRACT, code=Disassembly(code), concrete_storage=False)
        ws.put_account(acct)
        return ws, workloads.CONTRACT
    args, value = CONTRACTS[name]
    eng = symref.Engine()       # CODESIZE of a creation with arguments escapes: concrete on the oracle
    laser = LaserEVM(requires_statespace=False, device=device, strategy=BreadthFirstSearchStrategy, execution_timeout=0,
                     escape_handler=eng.step)
    ws = WorldState()
    creator = Account(CREATOR, balances=None)
    ws.put_account(creator)
    laser.open_states = [ws]
    execute_contract_creation(laser, None, CREATOR, CREATOR, workloads.bytecode(name) + args,
                              8_000_000, 1, value)
    assert len(laser.open_states) == 1, f"{name}: creation did not complete"
    out = laser.open_states[0]
    addr = next(a for a in out.accounts if a != CREATOR)
    return out, addr


def _outcomes_of_restatement(engine):
    out = Counter()
    for kind, s in engine.ended:
        c = tuple(x.raw for x in s.world_state.constraints)
        fn = s.environment.active_function_name
        if kind in ("stop", "return"):
            out[("txend", False, c, fn)] += 1
            out[("ws", c)] += 1
        elif kind == "exception":
            out[("txend", False, c, fn)] += 1
        elif kind == "revert":
            out[("txend", True, c, fn)] += 1
        elif kind == "end":
            out[("ws", c)] += 1
        else:
            out[(kind, c)] += 1
    return out


def run_both(device, name, monkeypatch):
    """(outcomes through LaserEVM + device, outcomes of the restatement, laser)."""
    monkeypatch.setattr(solver.args, "pruning_factor", 0)
    ws, addr = deploy(device, name)
    from copy import copy
    ws_ref = copy(ws)
    # --- batched LaserEVM: symbolic lanes on the device, escapes to the restatement
    handler_engine = symref.Engine()

    def handler(state):
        try:
            return handler_engine.step(state)
        except symref.Unsupported:
            handler_engine.ended.append(("unsupported", state))
            return []
    escaped = Counter()

    def counting_handler(state):
        ins = state.environment.code.instruction_list
        escaped.update([ins[state.mstate.pc]["opcode"] if state.mstate.pc < len(ins) else "END"])
        return handler(state)
    laser = LaserEVM(requires_statespace=False, device=device, strategy=BreadthFirstSearchStrategy, execution_timeout=0,
                     escape_handler=counting_handler)
    laser.escaped_ops = escaped
    got = Counter()
    laser.register_laser_hooks("transaction_end", lambda s, tx, ret, revert: got.update(
        [("txend", bool(revert), tuple(x.raw for x in s.world_state.constraints),
          s.environment.active_function_name)]))
    laser.register_laser_hooks("add_world_state", lambda s: got.update(
        [("ws", tuple(x.raw for x in s.world_state.constraints))]))
    laser.open_states = [ws]
    tx0 = int(tx_id_manager.get_next_tx_id())
    tx_id_manager.set_counter(tx0 - 1)
    execute_symbolic_message_call(laser, addr)
    got += _outcomes_of_restatement(handler_engine)
    # --- the restatement alone, from the same world state and transaction id
    tx_id_manager.set_counter(tx0 - 1)
    ref_engine = symref.Engine()
    txid = tx_id_manager.get_next_tx_id()
    sender = symbol_factory.BitVecSym(f"sender_{txid}", 256)
    acct = ws_ref[addr]
    tx = MessageCallTransaction(world_state=ws_ref, identifier=txid,
                                gas_price=symbol_factory.BitVecSym(f"gas_price{txid}", 256),
                                gas_limit=8_000_000, origin=sender, caller=sender, callee_account=acct,
                                call_data=SymbolicCalldata(txid),
                                call_value=symbol_factory.BitVecSym(f"call_value{txid}", 256))
    gs = tx.initial_global_state()
    gs.transaction_stack.append((tx, None))
    gs.world_state.transaction_sequence.append(tx)       # _setup_global_state_for_execution
    gs.world_state.constraints.append(
        Or(*[tx.caller == symbol_factory.BitVecVal(a, 256) for a in ACTORS.values()]))
    ref_engine.run([gs])
    return got, _outcomes_of_restatement(ref_engine), laser


# creation codes run by a symbolic creation (transaction/symbolic.py:154-200):
# constructor arguments are read past the end of the code from the symbolic
# calldata (CODESIZE + 0x200 pins its size, instructions.py:979-1104)
SYM_CREATIONS = ("symbolic_exec_bytecode.sol.o", "flag_array.sol.o")
# every reference code as a symbolic creation (round 4)
SYM_CREATIONS_ALL = list(SYM_CREATIONS) + [n for n in sorted(workloads.bytecode_names()) if n not in SYM_CREATIONS]


def _creation_tx(ws, code, txid):
    from mythril_amd.laser import ContractCreationTransaction, Disassembly, SymbolicCalldata
    return ContractCreationTransaction(
        world_state=ws, identifier=txid, gas_price=symbol_factory.BitVecSym(f"gas_price{txid}", 256),
        gas_limit=8_000_000, origin=CREATOR, code=Disassembly(code), caller=CREATOR,
        call_data=SymbolicCalldata(txid), call_value=symbol_factory.BitVecSym(f"call_value{txid}", 256))


def run_creation_both(device, name, monkeypatch):
    """(outcomes of a symbolic creation through LaserEVM + device, outcomes of
    the restatement, laser): every path's end with its constraint sequence."""
    from copy import copy
    from mythril_amd.laser import execute_symbolic_contract_creation
    monkeypatch.setattr(solver.args, "pruning_factor", 0)
    code = workloads.bytecode(name)
    ws0 = WorldState()
    ws0.put_account(Account(CREATOR, balances=None))
    ws_ref = copy(ws0)
    handler_engine = symref.Engine()

    def handler(state):
        try:
            return handler_engine.step(state)
        except symref.Unsupported:
            handler_engine.ended.append(("unsupported", state))
            return []
    escaped = Counter()

    def counting_handler(state):
        ins = state.environment.code.instruction_list
        escaped.update([ins[state.mstate.pc]["opcode"] if state.mstate.pc < len(ins) else "END"])
        return handler(state)
    laser = LaserEVM(requires_statespace=False, device=device, strategy=BreadthFirstSearchStrategy, execution_timeout=0,
                     escape_handler=counting_handler)
    laser.escaped_ops = escaped
    got = Counter()
    # a creation keeps its world state only when it returns code (svm.py:459-466):
    # path ends are compared by their transaction_end outcomes
    laser.register_laser_hooks("transaction_end", lambda s, tx, ret, revert: got.update(
        [("txend", bool(revert), tuple(x.raw for x in s.world_state.constraints),
          s.environment.active_function_name)]))
    tx0 = int(tx_id_manager.get_next_tx_id())
    tx_id_manager.set_counter(tx0 - 1)
    execute_symbolic_contract_creation(laser, code, world_state=ws0)
    tx_id_manager.set_counter(tx0 - 1)
    ref_engine = symref.Engine()
    txid = tx_id_manager.get_next_tx_id()
    tx = _creation_tx(ws_ref, code, txid)
    gs = tx.initial_global_state()
    gs.transaction_stack.append((tx, None))
    gs.world_state.transaction_sequence.append(tx)       # _setup_global_state_for_execution
    # transaction/symbolic.py:202-219: the caller is one of the actors
    gs.world_state.constraints.append(
        Or(*[tx.caller == symbol_factory.BitVecVal(a, 256) for a in ACTORS.values()]))
    ref_engine.run([gs])

    def ends(c):
        return Counter({k: v for k, v in c.items() if k[0] != "ws"})
    return ends(got + _outcomes_of_restatement(handler_engine)), ends(_outcomes_of_restatement(ref_engine)), laser
