"""C3 (BASELINE configs[2]) on the MI355X: ``myth analyze BECToken.sol -t N``
with every module -- tests/bectoken.py's assembled contract, kernels 1 and 2,
the exact procedure behind them -- printing the issue table, the SWC-101 at the
multiplication, the prefilter's share of the queries and the exact calls.

    python scripts/r06/c3_bec.py <tx_count> [--search] [--cpu]
"""
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import analyze  # noqa: E402
import bectoken  # noqa: E402
import fnames  # noqa: E402
from mythril_amd.laser.disassembly import SignatureDB  # noqa: E402


def main():
    n = int(sys.argv[1])
    d = tempfile.mkdtemp()
    fnames.signature_db(Path(d))
    os.environ["MYTHRIL_DIR"] = d
    SignatureDB._reset()
    if "--cpu" in sys.argv:
        from oracle_device import OracleDevice, OracleK2
        dev, k2 = OracleDevice(), OracleK2()
    else:
        from mythril_amd.device import GpuDevice
        dev = k2 = GpuDevice(0)
    t0 = time.perf_counter()
    issues, info = analyze.analyze("BECToken", None, n, dev, k2, code=bectoken.creation(),
                                   search="--search" in sys.argv)
    wall = time.perf_counter() - t0
    table = analyze.issue_table(issues)
    out = {"tx": n, "wall_s": wall, "issues": table, "mul_address": bectoken.mul_address(),
           "swc101_at_mul": any(r[0] == "101" and r[1] == bectoken.mul_address() and
                                r[2] == "batchTransfer(address[],uint256)" for r in table),
           **{k: info[k] for k in ("forks", "confirmations", "search", "fork_filter", "escapes_dropped", "exact",
                                   "cache", "lane_steps", "device_ms", "k2_ms", "kernel2_launches", "device_evals")}}
    print(json.dumps(out, default=str), flush=True)


if __name__ == "__main__":
    main()
