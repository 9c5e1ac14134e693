#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (the fields DESIGN.md quotes).
usage: bench_summary.py <bench.json>"""
import json
import sys


def main(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"C2 value {d['value'] / 1e9:.2f} G lane-steps/s, ms/step {d['ms_per_step']:.4f}, kernel {r['kernel_ms']:.4f} ms, "
          f"{r['bound']} frac {r['frac']:.3f}, traffic {r.get('traffic')}")
    for k in ("c2_unbucketed", "c2_two_streams", "c2_large_contract"):
        if k in d:
            print(f"{k} {d[k]['value'] / 1e9:.2f} G")
    c4 = d.get("constraint_evals") or {}
    if c4:
        print(f"C4 {c4['value'] / 1e9:.2f} G evals/s, roofline frac {c4['roofline']['frac']:.3f}, "
              f"without division charge {c4['roofline'].get('without_division_charge', {}).get('frac')}")
    h = d.get("hooked_c2")
    if h:
        print(f"hooked_c2 {h['lane_steps_per_s'] / 1e3:.1f} k lane-steps/s, wall {h['wall_s']:.2f} s, "
              f"launches {h['launches']}, hook events {h.get('hook_events')}")
    t = d.get("taint_c2")
    if t:
        print(f"taint_c2 device {t['device']['lane_steps_per_s'] / 1e3:.1f} k, host {t['host']['lane_steps_per_s'] / 1e3:.1f} k, "
              f"speedup {t['speedup']:.2f}")
    for k in ("symbolic_lanes", "taint_lanes"):
        x = d.get(k)
        if x:
            print(f"{k} {x['lane_steps_per_s'] / 1e9:.2f} G lane-steps/s, {x['lane_steps_per_launch']} steps in "
                  f"{x['kernel_ms']:.3f} ms, statuses {x['statuses']}")
    st = d.get("symbolic_tx")
    if st:
        for n, c in st["contracts"].items():
            print(f"symbolic_tx {n}: wall {c['wall_s']:.2f} s (k1 {c['kernel1_s'] * 1e3:.1f} ms, k2 {c['kernel2_s'] * 1e3:.1f} ms), "
                  f"{c['lane_steps']} lane-steps, forks {c['forks']}, open {c['open_states']}, queries {c['queries']}, "
                  f"hit {c['prefilter_hit_rate']:.3f} (lru {c['lru_hits']}, seed {c['seed_hits']}, unknown {c['unknown']}), "
                  f"k2 {c['constraint_evals_per_s_kernel'] / 1e6 if c['constraint_evals_per_s_kernel'] else 0:.0f} M evals/s, "
                  f"escapes dropped {c['escapes_dropped']}")
    cb = d.get("cpu_baseline")
    if cb:
        print(f"cpu_baseline {cb['value'] / 1e9:.3f} G on {cb['cores']} cores")


if __name__ == "__main__":
    main(sys.argv[1])
