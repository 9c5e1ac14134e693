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


def test_compact_line_fits_the_driver(tmp_path):
    """the driver keeps ~12 KB of output, so the one JSON
    line stays <= 4 KB with every contract key, the roofline and the CPU
    baseline -- checked on round 5's full record (23 KB, every field), and on a
    line bench.py prints on the oracle device."""
    import bench
    full = json.loads((HERE / "golden" / "bench_full_r05.json").read_text())
    line = bench.compact_line(full, "profiles/x.json")
    text = json.dumps(line)
    assert len(text) <= bench.LINE_LIMIT
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert line["fields"]["c4"]["roofline"]["frac"] > 0
    assert line["fields"]["myth_analyze"]["totals"]["issues"] == 26
    assert json.loads(text)["value"] == line["value"]


def test_bench_prints_one_compact_line_on_the_oracle_device(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rec = tmp_path / "full.json"
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(1, sys.argv[1:], script=%r))" %
            (str(ROOT), str(HERE / "bench_rank_cpu.py")))
    argv = ["--gpus", "1", "--steps", "2", "--warmup", "1", "--lanes", "128", "--no-c4", "--cpu-seconds", "0.2",
            "--rec-cap", "0", "--no-roofline", "--full-record", str(rec)]
    p = subprocess.run([sys.executable, "-c", code] + argv, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and len(lines[0]) <= 4096
    out = json.loads(lines[0])
    assert out["cpu_baseline"]["value"] > 0 and out["full_record"] == str(rec)
    assert json.loads(rec.read_text())["value"] == out["value"] or abs(
        json.loads(rec.read_text())["value"] / out["value"] - 1) < 1e-3
