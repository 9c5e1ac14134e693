"""Host profiles (cProfile, cumulative and internal time) of the LaserEVM bench
fields on the GPU box, one file per field: hooked_c2 and the device-action run
of taint_c2 (bench.py's own setup), written under the directory argv[1]."""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import bench  # noqa: E402
from mythril_amd.device import GpuDevice  # noqa: E402

out = Path(sys.argv[1])
out.mkdir(parents=True, exist_ok=True)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
which = sys.argv[3].split(",") if len(sys.argv) > 3 else ["hooked", "taint"]
dev = GpuDevice(0)


def prof(name, fn):
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    r = fn()
    pr.disable()
    wall = time.perf_counter() - t0
    buf = io.StringIO()
    buf.write(f"{name}: wall {wall:.3f} s under cProfile; result {r}\n")
    pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(50)
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(40)
    (out / f"{name}.txt").write_text(buf.getvalue())
    print(name, wall, flush=True)


def taint_device():
    import refmodules
    from refmodules import hooks_of
    from mythril_amd.laser import LaserEVM
    from mythril_amd.laser.strategy import BreadthFirstSearchStrategy
    names = ("IntegerArithmetics", "TxOrigin", "ArbitraryStorage", "ArbitraryJump", "UserAssertions",
             "Exceptions", "StateChangeAfterCall")
    laser = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy, execution_timeout=0)
    laser.track_objects = True
    mods = [getattr(refmodules, m)() for m in names]
    laser.register_hooks("pre", hooks_of(mods, "pre"))
    laser.register_hooks("post", hooks_of(mods, "post"))
    bench._c2_laser_states(laser, n, bench.workloads_seed(0))
    t0 = time.perf_counter()
    laser.exec()
    wall = time.perf_counter() - t0
    return {"lane_steps": laser.lane_steps, "wall_s": wall, "lane_steps_per_s": laser.lane_steps / wall,
            "launches": laser.launches, "issues": sum(len(m.issues) for m in mods)}


if "hooked" in which:
    prof("hooked_c2", lambda: bench.run_hooked_c2(dev, n, 0))
if "taint" in which:
    prof("taint_c2_device", taint_device)
