"""Host profile (cProfile) of bench.py's myth_analyze field on the GPU (the 18
contracts, -t 2, all modules; no CPU comparator):
    python scripts/r05/prof_analyze.py OUT.txt"""
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
dev = GpuDevice(0)
bench.run_myth_analyze(dev, 2, cpu=False)          # warm-up
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
r = bench.run_myth_analyze(dev, 2, cpu=False)
pr.disable()
wall = time.perf_counter() - t0
buf = io.StringIO()
buf.write(f"myth_analyze: wall {wall:.3f} s under cProfile; job_wall_s {r['job_wall_s']:.3f}, "
          f"host_fraction {r['host_fraction']:.3f}\n")
for n, row in sorted(r["contracts"].items(), key=lambda kv: -kv[1]["wall_s"]):
    buf.write(f"  {n}: {row['wall_s']:.3f} s (k1 {row['kernel1_s']:.4f}, k2 {row['kernel2_s']:.4f})\n")
pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(80)
pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(50)
out.parent.mkdir(parents=True, exist_ok=True)
out.write_text(buf.getvalue())
print("myth_analyze", wall, flush=True)
