"""Round 5 diagnostic: myth analyze -f <code> -t 2 (all modules) on the device
and on the C oracles, per contract: issues, confirmations, escapes, forks."""
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import analyze  # noqa: E402
import fnames  # noqa: E402
from mythril_amd.laser.disassembly import SignatureDB  # noqa: E402
from oracle_device import OracleDevice, OracleK2  # noqa: E402

names = sys.argv[1].split(",")
gpu = "--gpu" in sys.argv
d = tempfile.mkdtemp()
fnames.signature_db(Path(d))
os.environ["MYTHRIL_DIR"] = d
SignatureDB._reset()
devs = [("cpu", OracleDevice(), OracleK2())]
if gpu:
    from mythril_amd.device import GpuDevice
    g = GpuDevice(0)
    devs.append(("gpu", g, g))
mods = [None] + [m for m in sys.argv[2:] if not m.startswith("--")]
for name in names:
  for mod in mods:
    for tag, dev, k2 in devs:
        issues, info = analyze.analyze(name, mod, 2, dev, k2)
        print(tag, name, mod, analyze.issue_table(issues), {k: info[k] for k in (
            "lane_steps", "launches", "forks", "escapes_dropped", "confirmations", "fork_filter")}, flush=True)
