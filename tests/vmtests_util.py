"""Shared helpers: turn the reference's VMTests vectors (tests/golden/vmtests.json) into
lane images and judge a lane's outcome exactly as the reference harness does
(tests/laser/evm_testsuite/evm_test.py:110-189 of the reference)."""
import json
from pathlib import Path

from mythril_amd.lanes import (LaneBatch, LaneShape, MG_ESCAPE, MG_HOOK, MG_RUNNING,
                               WORLD_STATE_KEPT)

GOLDEN = Path(__file__).resolve().parent / "golden"


def load_vmtests():
    return json.loads((GOLDEN / "vmtests.json").read_text())


def load_json(name):
    return json.loads((GOLDEN / name).read_text())


def account(accounts: dict, address: str):
    """Look an account up by numeric address (fixture keys keep leading zeros)."""
    want = int(address, 16)
    for k, det in accounts.items():
        if int(k, 16) == want:
            return det
    return None


def vm_shape(vectors, n=None):
    cd = max([len(v["data"]) // 2 for v in vectors] + [32])
    st = max([len((account(v["pre"], v["address"]) or {}).get("storage", {}))
              for v in vectors] + [0])
    return LaneShape(n=n or len(vectors), stack_cap=1024, mem_cap=1 << 20,
                     calldata_cap=(cd + 31) // 32 * 32, storage_cap=max(64, st + 32))


def fill_lane(batch: LaneBatch, i: int, v: dict, code_id: int):
    """transaction/concolic.py:75-122 with the VMTests harness' arguments
    (evm_test.py:136-152): concrete caller/origin/value/gasprice, gas_limit = exec.gas,
    pre-state storage of the callee as concrete storage (K(0) + stores)."""
    pre = account(v["pre"], v["address"]) or {"storage": {}}
    storage = {int(k, 16): int(val, 16) for k, val in pre["storage"].items()}
    batch.set_lane(i, code_id=code_id, calldata=bytes.fromhex(v["data"]),
                   address=int(v["address"], 16), caller=int(v["caller"], 16),
                   origin=int(v["origin"], 16), callvalue=int(v["value"], 16),
                   gasprice=int(v["gas_price"], 16), gas_limit=v["gas"], storage=storage)


def judge(batch: LaneBatch, i: int, v: dict):
    """Return (verdict, detail): verdict in {"pass", "fail", "escaped"}.

    evm_test.py:153-189:
      * if the vector has a gas figure below the block gas limit, the final
        state's min gas must be <= gas used and min <= max;
      * post == {}  => no open world state (exception, revert, out of gas, ...);
      * post != {}  => exactly one open world state whose listed storage keys hold
        the listed values.
    """
    st = int(batch.status[i])
    if st in (MG_ESCAPE, MG_HOOK, MG_RUNNING):
        return "escaped", f"status={st} aux={int(batch.aux[i]):#x}"
    gas_used = v["gas_used"]
    if gas_used is not None and gas_used < v["block_gas_limit"]:
        gmin, gmax = int(batch.gas_min[i]), int(batch.gas_max[i])
        if not (gmin <= gmax and gmin <= gas_used):
            return "fail", f"gas ({gmin},{gmax}) vs used {gas_used}"
    open_state = st in WORLD_STATE_KEPT
    if not v["post"]:
        return ("pass", "") if not open_state else ("fail", f"expected no open state, got {st}")
    if not open_state:
        return "fail", f"expected an open state, got status {st} aux {int(batch.aux[i])}"
    for addr, det in v["post"].items():
        if int(addr, 16) == int(v["address"], 16):
            storage = batch.storage_dict(i, drop_zero=False)
        else:  # accounts the lane cannot touch keep their pre-state storage
            pre = account(v["pre"], addr) or {"storage": {}}
            storage = {int(k, 16): int(x, 16) for k, x in pre["storage"].items()}
        for k, val in det["storage"].items():
            got = storage.get(int(k, 16), 0)
            if got != int(val, 16):
                return "fail", f"storage[{k}] = {got:#x}, expected {val}"
    return "pass", ""
