"""Host profile (cProfile) of bench.py's symbolic_tx field, one contract.

    python scripts/r05/prof_symtx.py OUT.txt [contract] [replicas] [gpu|oracle]

`oracle` runs it in this container on the CPU restatements of both kernels
(tests/oracle_device.py), so the host layer can be profiled without a GPU; the
oracle's own time shows up under oracle_device / oracle.* and is not host work.
"""
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
import symref  # noqa: E402

out = Path(sys.argv[1])
name = sys.argv[2] if len(sys.argv) > 2 else "exceptions.sol.o"
replicas = int(sys.argv[3]) if len(sys.argv) > 3 else 8
kind = sys.argv[4] if len(sys.argv) > 4 else "gpu"
if kind == "gpu":
    from mythril_amd.device import GpuDevice
    dev = GpuDevice(0)
else:
    from oracle_device import OracleDevice, OracleK2

    class _Both(OracleDevice):
        def __init__(self):
            super().__init__()
            self._k2 = OracleK2()

        def eval(self, prog, pool):
            return self._k2.eval(prog, pool)

        def eval_bits(self, prog, pool):
            return self._k2.eval_bits(prog, pool)

    dev = _Both()
bench.SYMBOLIC_TX_CODES = (name,)
handler = symref.Engine(signals=True).step
bench.run_symbolic_tx(dev, replicas, 2, 1024, handler)      # warm-up (compiles, caches)
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
r = bench.run_symbolic_tx(dev, replicas, 2, 1024, handler)
pr.disable()
wall = time.perf_counter() - t0
row = r["contracts"][name]
buf = io.StringIO()
buf.write(f"{name} x{replicas} on {kind}: wall {wall:.3f} s under cProfile; field wall {row['wall_s']:.3f} s, "
          f"forks {row['forks']}, lane_steps {row['lane_steps']}\n")
pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(70)
pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(50)
out.parent.mkdir(parents=True, exist_ok=True)
out.write_text(buf.getvalue())
print(name, kind, wall, row["wall_s"], flush=True)
