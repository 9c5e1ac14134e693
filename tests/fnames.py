"""Test helpers for the function table and active_function_name (no GPU).

* ``easm_from_table``: asm.instruction_list_to_easm (asm.py:38-52) rendered from
  a code table (opcode byte and address per instruction, as the device's
  mg_code_table or the oracle's code_table return it) plus the code's bytes for
  the PUSH arguments (asm.py:136-142: the bytes present, cut at the end).
* ``signature_db``: a SignatureDB file (support/signatures.py schema) holding
  the text signatures of tests/golden/signatures.json, as the reference's
  ``~/.mythril/signatures.db`` would after ``import_solidity_file``.
* ``names_by_single_step``: the reference's exec loop for one concrete path,
  one instruction per oracle call, with _new_node_state's switch
  (svm.py:549-637) applied after every JUMP / JUMPI from the host
  Disassembly's table -- the restatement the device's per-lane function-entry
  record (mg_lane_soa.fent) is checked against.
"""
from __future__ import annotations

import json
import sqlite3
from pathlib import Path

from mythril_amd.keccak import keccak256
from mythril_amd.laser.disassembly import SignatureDB
from mythril_amd.laser.opcodes import ADDRESS_OPCODE_MAPPING, push_width

GOLDEN = Path(__file__).resolve().parent / "golden"
SIGNATURES = json.loads((GOLDEN / "signatures.json").read_text())


def easm_from_table(ops, addrs, code: bytes) -> str:
    out = []
    for op, a in zip(ops.tolist(), addrs.tolist()):
        name = ADDRESS_OPCODE_MAPPING.get(op, "INVALID")
        line = f"{a} {name}"
        w = push_width(name)
        if w:
            line += " 0x" + code[a + 1: a + 1 + w].hex()
        out.append(line + "\n")
    return "".join(out)


def selector(text_sig: str) -> str:
    return "0x" + keccak256(text_sig.encode())[:4].hex()


def signature_db(directory: Path) -> Path:
    """Write <directory>/signatures.db with every fixture signature."""
    directory.mkdir(parents=True, exist_ok=True)
    path = directory / "signatures.db"
    with sqlite3.connect(path) as conn:
        conn.execute("CREATE TABLE IF NOT EXISTS signatures(byte_sig VARCHAR(10), text_sig VARCHAR(255),"
                     "PRIMARY KEY (byte_sig, text_sig))")
        for sigs in SIGNATURES.values():
            for t in sigs:
                conn.execute("INSERT OR IGNORE INTO signatures VALUES (?,?)", (selector(t), t))
    return path


def use_signature_db(monkeypatch, tmp_path: Path) -> None:
    """MYTHRIL_DIR -> a fresh directory holding the fixture signature database."""
    signature_db(tmp_path)
    monkeypatch.setenv("MYTHRIL_DIR", str(tmp_path))
    SignatureDB._reset()


def names_by_single_step(oracle, batch, i: int, disassembly, start_name: str = "fallback",
                         max_steps: int = 100_000) -> str:
    """Step lane i of `batch` (an oracle image) one instruction at a time and
    return the function name the reference's exec loop leaves on its last
    state: after a JUMP / JUMPI that executed (the lane is still running, or it
    ran into its next stop after the jump), the successor's address switches
    the name as _new_node_state does."""
    from mythril_amd.lanes import MG_RUNNING
    instrs = disassembly.instruction_list
    name = start_name
    for _ in range(max_steps):
        if int(batch.status[i]) != MG_RUNNING:
            break
        pc0 = int(batch.pc[i])
        steps0 = int(batch.steps[i])
        op = instrs[pc0]["opcode"] if pc0 < len(instrs) else None
        oracle.run(batch, i, 1, max_steps=1)
        executed = int(batch.steps[i]) > steps0
        if op in ("JUMP", "JUMPI") and executed and int(batch.status[i]) == MG_RUNNING:
            pc = int(batch.pc[i])
            if pc < len(instrs):
                address = instrs[pc]["address"]
                if address in disassembly.address_to_function_name:
                    name = disassembly.address_to_function_name[address]
                elif address == 0:
                    name = "fallback"
    return name
