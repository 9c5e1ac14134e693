"""Diagnose the graph run (requires_statespace) of one analysis_tests row on
the MI355X: prints every 200th popped state (pc, opcode, depth, work list)
and stops after a step cap, so a run that stops advancing shows where."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import analyze  # noqa: E402
from mythril_amd.laser import svm  # noqa: E402

name, module, tx = sys.argv[1], sys.argv[2], int(sys.argv[3])
cap = int(sys.argv[4]) if len(sys.argv) > 4 else 20000
dev_kind = sys.argv[5] if len(sys.argv) > 5 else "gpu"
orig = svm.LaserEVM._host_only
count = [0]
t0 = time.time()


def probe(self, states, final_states, track_gas):
    count[0] += 1
    s = states[0]
    if count[0] % 200 == 0 or count[0] > cap:
        print(f"{count[0]} t={time.time() - t0:.1f}s pc={s.mstate.pc} op={svm._opcode_at(s)} "
              f"depth={s.mstate.depth} wl={len(self.work_list)} id={id(s)}", flush=True)
    if count[0] > cap + 20:
        raise SystemExit("step cap")
    return orig(self, states, final_states, track_gas)


svm.LaserEVM._host_only = probe
from mythril_amd import device as devmod  # noqa: E402
_step = devmod.GpuDevice.step


def step(self, *a, **k):
    st = _step(self, *a, **k)
    if count[0] > cap - 3:
        b = self._batch if hasattr(self, "_batch") else None
        print("  step", k, st, flush=True)
    return st


devmod.GpuDevice.step = step
_dl = devmod.GpuDevice.download_range


def download_range(self, b, lo, cnt, live=False):
    out = _dl(self, b, lo, cnt, live=live)
    if count[0] > cap - 3:
        print("  lane0", {f: int(getattr(b, f)[0]) for f in ("pc", "sp", "status", "aux", "steps", "flags", "code_id")},
              "sym" if hasattr(b, "node") else "", b.shape, flush=True)
    return out


devmod.GpuDevice.download_range = download_range
if dev_kind == "gpu":
    from mythril_amd.device import GpuDevice
    d = GpuDevice(0)
    k2 = d
else:
    from oracle_device import OracleDevice, OracleK2
    d, k2 = OracleDevice(), OracleK2()
issues, info = analyze.analyze(name, module, tx, d, k2, statespace=True)
print("done", count[0], f"{time.time() - t0:.1f}s", analyze.issue_table(issues))
