"""The headline kernels' launches in a rocprofv3 kernel trace of bench.py:

    python scripts/r06/headline_launches.py TRACE.csv OUT.json

k_lane_step (no loop bound) at the C2 grid (65,536 lanes) and k_bv_eval at the
C4 grid.  The C2 grid is launched by several fields (unbucketed order, the timed
batches, two streams, the roofline pass); the timed region is the run of
`warmup + steps` consecutive launches on one queue that follows the unbucketed
field's launches, so besides every launch at that grid the file gives that run's
average (the figure `roofline.kernel_ms` must agree with)."""
import csv
import json
import statistics
import sys


def stats(ms):
    return {"launches": len(ms), "avg_ms": statistics.fmean(ms), "median_ms": statistics.median(ms),
            "min_ms": min(ms), "max_ms": max(ms)} if ms else {"launches": 0}


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    c2 = [r for r in rows if r["Kernel_Name"].startswith("void k_lane_step<false>") and int(r["Grid_Size_X"]) == 65536]
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in c2]
    bv = [r for r in rows if r["Kernel_Name"].startswith("k_bv_eval")]
    big = max((int(r["Grid_Size_X"]) for r in bv), default=0)
    c4 = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in bv if int(r["Grid_Size_X"]) == big]
    # bench.py defaults: 1 + 10 unbucketed launches, then 3 warm-up + 20 timed
    unb, warm, steps = 11, 3, 20
    timed = ms[unb + warm: unb + warm + steps]
    out = {"k_lane_step_c2": {"grid": 65536, **stats(ms)},
           "k_lane_step_c2_timed_run": {"launch_index": [unb + warm, unb + warm + steps], **stats(timed)},
           "k_bv_eval_c4": {"grid": big, **stats(c4)}}
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
