"""bench.py --gpus N starts N ranks itself (bench.launch_ranks) when WORLD_SIZE is
unset.  On CPU: 2 gloo ranks with the oracle device; the one JSON line reports
n_gpus == 2, weak scaling, and the whole-job lane-steps of both ranks."""
import json
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent


def test_two_ranks_from_the_bench_entry():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(2, sys.argv[1:], script=%r))" %
            (str(ROOT), str(HERE / "bench_rank_cpu.py")))
    argv = ["--gpus", "2", "--steps", "2", "--warmup", "1", "--lanes", "128", "--no-c4",
            "--no-cpu-baseline", "--no-roofline", "--rec-cap", "0"]
    p = subprocess.run([sys.executable, "-c", code] + argv, env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    per_rank = out["config"]["lane_steps_per_batch"]
    # whole-job value = both ranks' lane-steps / the slower rank's time
    assert out["value"] > 0 and out["value"] * out["ms_per_step"] / 1e3 > 1.5 * per_rank


def test_launcher_returns_worst_status(tmp_path):
    import bench
    bad = tmp_path / "fail_rank.py"
    bad.write_text("import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert bench.launch_ranks(2, [], script=str(bad)) == 3
