#!/usr/bin/env python3
"""Headline benchmark: EVM lane-steps/s of the batched LASER core (BASELINE.json).

Workload (configs[1]): 65,536 concrete lanes per GPU stepping token.sol's
runtime (precompiled overflow.sol.o, see mythril_amd/workloads.py) with random
calldata.  One step = one batch: reset every lane from its
resident initial image (calldata, env, storage already in HBM) and run the
stepping kernel until every lane has halted; the timed batches are enqueued
back to back on the library's stream (mg_run_batches) with one host wait.  Weak scaling: every rank runs its
own 65,536 lanes (seed + rank); the only collective is the coverage all-gather
after the timed region's batches (§8(e)), over RCCL.

Prints ONE JSON line (rank 0).

Multi-GPU: `python bench.py --gpus N` with no WORLD_SIZE in the environment
starts N rank processes itself (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE set,
rendezvous on 127.0.0.1) before anything touches a GPU, and exits with their
status; under torch.distributed.run (WORLD_SIZE set) it is one of the ranks.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--lanes", type=int, default=65536)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--c4-dags", type=int, default=1_000_000)
    ap.add_argument("--c4-models", type=int, default=4096)
    ap.add_argument("--c4-steps", type=int, default=3)
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--rec-cap", type=int, default=128,
                    help="function-manager record words per lane (0: registrations off)")
    ap.add_argument("--profile-only", action="store_true",
                    help="run warmup+steps with no JSON extras (for rocprofv3)")
    ap.add_argument("--hooked-lanes", type=int, default=4096,
                    help="lanes of the hooked-C2 field (0: off): C2 through LaserEVM with the "
                         "default detection modules' opcode hooks registered")
    ap.add_argument("--overlap-steps", type=int, default=40,
                    help="batches per stream of the C2 lanes on two library contexts at once, "
                         "reported as c2_two_streams (0: off)")
    ap.add_argument("--unbucketed-steps", type=int, default=10,
                    help="batches of the C2 lanes in generation order, reported as c2_unbucketed (0: off)")
    ap.add_argument("--large-steps", type=int, default=10,
                    help="batches of the large-contract field (c2_large_contract; 0: off)")
    ap.add_argument("--taint-lanes", type=int, default=4096,
                    help="lanes of the taint_c2 field (0: off): C2 through LaserEVM with the integer "
                         "and TxOrigin modules' hooks as device actions (taint lanes) and on the host")
    ap.add_argument("--symbolic-lanes", type=int, default=65536,
                    help="symbolic lanes for the k_sym_step field (0: skip)")
    ap.add_argument("--symbolic-replicas", type=int, default=2,
                    help="replicas of each contract in the symbolic_tx field (0: off; 8 until round 5, "
                         "when its unknown fork verdicts were kept: the exact procedure's host time "
                         "grows faster than the replicas)")
    ap.add_argument("--symbolic-tx", type=int, default=2, help="transactions of the symbolic_tx field (-t)")
    ap.add_argument("--analyses", type=int, default=2,
                    help="transactions (-t) of the 18-contract analyses field (0: skip)")
    ap.add_argument("--seed-models", type=int, default=1024,
                    help="witness seed models beside the LRU cache in the symbolic_tx field")
    ap.add_argument("--taint-modes", default="device,host",
                    help="taint_c2 modes to run (device: batch-safe hooks on kernel 1; host: as host events)")
    ap.add_argument("--host-profile", default=None,
                    help="directory: cProfile the LaserEVM fields (hooked_c2, taint_c2, symbolic_tx) "
                         "and write each one's cumulative-time table there")
    ap.add_argument("--c3-tx", type=int, default=1,
                    help="transactions of the C3 field (BECToken, all modules); 0 skips it.  -t 1 holds "
                         "the CVE-2018-10299 finding (3 s on the MI355X); -t 2 takes about a minute, "
                         "most of it in the exact procedure (profiles/r06/README.md)")
    ap.add_argument("--full-record", default="gpurun_out/bench_full.json",
                    help="where the whole record goes (stdout carries the compact line, <= 4 KB)")
    ap.add_argument("--no-roofline", action="store_true",
                    help="skip the profiling pass behind `roofline` (CPU rehearsals of the rank launcher)")
    return ap.parse_args(argv)


def _log(rank: int, what: str) -> None:
    """Progress on stderr (the JSON line stays alone on stdout)."""
    if rank == 0:
        print(f"bench.py: {what} [{time.strftime('%H:%M:%S')}]", file=sys.stderr, flush=True)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv, script: str = None) -> int:
    """Start one rank process per GPU (RANK = LOCAL_RANK = k, WORLD_SIZE = n,
    MASTER_ADDR 127.0.0.1) and wait for all; returns the worst exit status.
    The parent never initialises a GPU: it only spawns and waits."""
    import subprocess
    port = _free_port()
    procs = []
    for k in range(n):
        env = dict(os.environ, RANK=str(k), LOCAL_RANK=str(k), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, script or str(Path(__file__).resolve())] + list(argv),
                                      env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main(argv=None, device_factory=None, backend: str = "nccl"):
    """One rank of the benchmark.  device_factory(local_rank) -> device (default
    GpuDevice); backend: the torch.distributed backend for world > 1 (nccl =
    RCCL over xGMI on the GPU box)."""
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:] if argv is None else argv))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if rank == 0:
        # a liveness line while a long host-side field (an exact query, a
        # transaction round) runs: a minute of silence reads as a hang
        import threading

        def _beat():
            while True:
                time.sleep(60)
                _log(0, "running")
        threading.Thread(target=_beat, daemon=True).start()
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting n_gpus={world}",
              file=sys.stderr)
    import torch
    import torch.distributed as dist

    dist_on = world > 1
    gpu = device_factory is None
    if dist_on:
        if gpu:
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from mythril_amd import workloads
    from mythril_amd import roofline

    if gpu:
        from mythril_amd.device import GpuDevice
        dev = GpuDevice(local)
    else:
        dev = device_factory(local)
    from mythril_amd import dist as mdist

    def barrier():
        if dist_on:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    code = workloads.bytecode("overflow.sol.o")
    cid = dev.load_code(code)
    batch = workloads.c2_batch(args.lanes, code_id=cid, seed=workloads.C2_SEED + rank,
                               stack_cap=1024, mem_cap=1024, rec_cap=args.rec_cap)
    # lanes bucketed by (code, selector, calldata length) so a wavefront walks
    # one function's path (mythril_amd/lanes.py:bucket_order); parity of every
    # lane is independent of its position in the batch
    from mythril_amd.lanes import bucket_order, permuted
    dev.alloc(batch.shape, coverage=True)
    unbucketed = None
    if args.unbucketed_steps and not args.profile_only:
        # the same lanes in generation order: what bucketing buys (reported
        # beside `value`, never as it)
        _log(rank, "C2 unbucketed")
        dev.upload(workloads.slim_copy(batch))
        dev.run_batches(1)
        barrier()
        t0 = time.perf_counter()
        ust = dev.run_batches(args.unbucketed_steps)
        barrier()
        uel = time.perf_counter() - t0
        uel, usteps = mdist.reduce_timing(uel, float(sum(st.lane_steps for st in ust)))
        unbucketed = {"value": usteps / uel, "unit": "lane-steps/s",
                      "ms_per_step": 1000.0 * uel / args.unbucketed_steps,
                      "kernel_ms_per_batch": float(np.mean([st.kernel_ms for st in ust])),
                      "order": "generation order (no bucket_order)"}
    batch = permuted(batch, bucket_order(batch))
    dev.upload(workloads.slim_copy(batch))
    _log(rank, "C2 bucketed (timed)")

    if args.warmup:
        dev.run_batches(args.warmup)

    # the K batches are enqueued back to back (reset + stepping launch each,
    # mg_run_batches) with one host wait: no host round trip between batches
    barrier()
    t0 = time.perf_counter()
    stats = dev.run_batches(args.steps) if args.steps else []
    lane_steps = sum(st.lane_steps for st in stats)
    kernel_ms = [st.kernel_ms for st in stats]
    if any(st.running for st in stats):
        raise RuntimeError("a C2 batch ended with lanes still running")
    barrier()
    elapsed = time.perf_counter() - t0

    # coverage all-gather over RCCL (coverage_plugin.py semantics: OR of bits)
    cov_union = mdist.allgather_coverage(dev.coverage(cid))
    elapsed, total_steps = mdist.reduce_timing(elapsed, float(lane_steps))
    total_steps = int(total_steps)

    overlap = None
    if args.overlap_steps and gpu and not args.profile_only:
        _log(rank, "C2 on two streams")
        overlap = run_two_streams(dev, batch, code, args.overlap_steps, local, barrier)

    large = None
    if args.large_steps and not args.profile_only:
        _log(rank, "C2 on the 3,523-instruction fixture")
        large = run_large(dev, args, rank, barrier)
        # back to the C2 batch for the roofline profile below
        dev.alloc(batch.shape, coverage=True)
        dev.upload(workloads.slim_copy(batch))

    roof = None
    if rank == 0 and not args.profile_only and not args.no_roofline:
        _log(rank, "C2 roofline profile")
        roof = roofline.lane_step_roofline(dev, batch, cid, kernel_ms=float(np.mean(kernel_ms)) if kernel_ms else 0.0)

    def host_profiled(name, fn):
        """fn(), under cProfile when --host-profile is set (rank 0)."""
        if not args.host_profile or rank != 0:
            return fn()
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        try:
            return fn()
        finally:
            pr.disable()
            os.makedirs(args.host_profile, exist_ok=True)
            buf = io.StringIO()
            pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(60)
            pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(40)
            Path(args.host_profile, f"{name}.txt").write_text(buf.getvalue())

    hooked = None
    if args.hooked_lanes and gpu and not args.profile_only:
        _log(rank, f"hooked C2 ({args.hooked_lanes} lanes)")
        hooked = host_profiled("hooked_c2", lambda: run_hooked_c2(dev, args.hooked_lanes, rank))

    taint = None
    if args.taint_lanes and gpu and not args.profile_only:
        _log(rank, f"taint C2 ({args.taint_lanes} lanes)")
        taint = host_profiled("taint_c2", lambda: run_taint_c2(dev, args.taint_lanes, rank,
                                                                  tuple(args.taint_modes.split(","))))

    symlanes = None
    if args.symbolic_lanes and gpu and not args.profile_only:
        _log(rank, f"symbolic lanes ({args.symbolic_lanes}) on k_sym_step")
        symlanes = run_symbolic_lanes(dev, args.symbolic_lanes)

    taintlanes = None
    if args.symbolic_lanes and gpu and not args.profile_only:
        _log(rank, f"taint lanes ({args.symbolic_lanes}) on k_sym_step")
        taintlanes = run_taint_lanes(dev, args.symbolic_lanes, rank)

    symb = None
    if args.symbolic_replicas and gpu and not args.profile_only:
        _log(rank, f"symbolic transactions (-t {args.symbolic_tx}, {args.symbolic_replicas} replicas)")
        sys.path.insert(0, str(ROOT / "tests"))
        import symref
        symb = host_profiled("symbolic_tx", lambda: run_symbolic_tx(
            dev, args.symbolic_replicas, args.symbolic_tx, args.seed_models, log=lambda m: _log(rank, m),
            escape_handler=symref.Engine(signals=True).step))

    analyses = None
    if args.analyses and gpu and not args.profile_only:
        _log(rank, f"myth analyze over the 18 contracts (-t {args.analyses})")
        analyses = host_profiled("myth_analyze", lambda: run_myth_analyze(
            dev, args.analyses, log=lambda m: _log(rank, m), cpu=not args.no_cpu_baseline))

    c3 = None
    if args.c3_tx and gpu and not args.profile_only and rank == 0:
        c3 = host_profiled("c3_bectoken", lambda: run_c3_bectoken(dev, args.c3_tx, log=lambda m: _log(rank, m)))

    c4 = None
    if not args.no_c4:
        _log(rank, "C4")
        c4 = run_c4(args, dev, rank, world, barrier, dist_on)

    if rank == 0 and not args.profile_only:
        value = total_steps / elapsed
        steps_per_batch = lane_steps / max(args.steps, 1)
        kms = float(np.mean(kernel_ms)) if kernel_ms else 0.0
        if roof and roof.get("issue_floor") and kms > 0:
            fl = roof["issue_floor"]
            fl["ceiling_lane_steps_per_s"] = steps_per_batch / (kms / 1e3) / fl["busy_frac"]
            fl["frac"] = (total_steps / elapsed / world) / fl["ceiling_lane_steps_per_s"]
        out = {
            "metric": "EVM lane-steps/s (kernel 1, C2: 65,536 concrete lanes/GPU, token.sol runtime)",
            "value": value,
            "unit": "lane-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / max(args.steps, 1),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32x8 (256-bit integer)",
            "data": "synthetic calldata (PCG64 seed 0x4D595448 + rank), precompiled overflow.sol.o",
            "config": {"workload": "C2: 65,536 concrete lanes/GPU stepping token.sol runtime "
                                   "(overflow.sol.o) with random calldata",
                       "lanes_per_gpu": args.lanes, "lane_steps_per_batch": steps_per_batch,
                       "kernel_ms_per_batch": kms,
                       "coverage_instructions": int(cov_union.sum()),
                       "function_manager_records": args.rec_cap > 0,
                       "parallelism": f"lanes sharded x{world}, RCCL coverage all-gather"},
            "roofline": roof,
        }
        if unbucketed is not None:
            out["c2_unbucketed"] = unbucketed
        if overlap is not None:
            out["c2_two_streams"] = overlap
        if large is not None:
            out["c2_large_contract"] = large
        if not args.no_cpu_baseline:
            from oracle import cpu_baseline
            _log(rank, "C2 CPU baseline")
            out["cpu_baseline"] = cpu_baseline.c2_lane_steps(code, args.cpu_seconds)
        if c4 is not None:
            if not args.no_cpu_baseline:
                from oracle import cpu_baseline
                _log(rank, "C4 CPU baseline")
                c4["cpu_baseline"] = cpu_baseline.c4_evals(args.c4_models, args.cpu_seconds)
            out["constraint_evals"] = c4
        if hooked is not None:
            out["hooked_c2"] = hooked
        if taint is not None:
            out["taint_c2"] = taint
        if symlanes is not None:
            out["symbolic_lanes"] = symlanes
        if taintlanes is not None:
            out["taint_lanes"] = taintlanes
        if symb is not None:
            out["symbolic_tx"] = symb
        if analyses is not None:
            out["myth_analyze"] = analyses
        if c3 is not None:
            out["c3_bectoken"] = c3
        full = Path(args.full_record)
        try:
            full.parent.mkdir(parents=True, exist_ok=True)
            full.write_text(json.dumps(out, indent=1) + "\n")
        except OSError as e:
            _log(rank, f"full record not written ({e})")
        print(json.dumps(compact_line(out, str(args.full_record))), flush=True)
    if dist_on:
        dist.destroy_process_group()


LINE_LIMIT = 4096


def _r(x, digits: int = 4):
    """Floats to `digits` significant digits (the compact line's size)."""
    if isinstance(x, float):
        return float(f"{x:.{digits}g}")
    if isinstance(x, dict):
        return {k: _r(v, digits) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_r(v, digits) for v in x]
    return x


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def compact_line(out: dict, full_record: str) -> dict:
    """The one JSON line the driver reads (at most LINE_LIMIT bytes): the
    contract keys, the headline roofline and CPU baseline, and a summary of
    every secondary field; the whole record goes to `full_record`."""
    line = _pick(out, ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                       "higher_is_better", "scaling", "vs_baseline", "dtype", "data"))
    line["config"] = _pick(out.get("config", {}), ("workload", "lanes_per_gpu", "lane_steps_per_batch",
                                                   "kernel_ms_per_batch", "parallelism"))
    roof = out.get("roofline")
    if roof:
        line["roofline"] = _pick(roof, ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel",
                                        "kernel_ms", "priced_as", "traffic_frac", "frac_sustained"))
        if "alt" in roof:
            line["roofline"]["alt"] = _pick(roof["alt"], ("bound", "frac"))
    else:
        line["roofline"] = None
    cb = out.get("cpu_baseline")
    line["cpu_baseline"] = (_pick(cb, ("value", "unit", "cores", "kind", "sample", "single_core_value",
                                       "usable_cores")) if cb else None)
    f = {}
    c4 = out.get("constraint_evals")
    if c4:
        f["c4"] = _pick(c4, ("value", "unit", "ms_per_step", "scaling"))
        if c4.get("roofline"):
            f["c4"]["roofline"] = _pick(c4["roofline"], ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                         "frac_sustained"))
        if c4.get("cpu_baseline"):
            f["c4"]["cpu_baseline"] = _pick(c4["cpu_baseline"], ("value", "cores", "kind"))
    for k in ("c2_unbucketed", "c2_two_streams", "c2_large_contract"):
        if out.get(k):
            f[k] = out[k].get("value")
    if out.get("hooked_c2"):
        f["hooked_c2"] = out["hooked_c2"].get("lane_steps_per_s")
    if out.get("taint_c2"):
        t = out["taint_c2"]
        f["taint_c2"] = {m: t[m].get("lane_steps_per_s") for m in ("device", "host") if isinstance(t.get(m), dict)}
    for k in ("symbolic_lanes", "taint_lanes"):
        v = out.get(k)
        if v:
            f[k] = {"value": v.get("lane_steps_per_s"), "steps_per_lane": (v.get("lane_steps_per_launch", 0) /
                                                                           max(v.get("lanes", 1), 1)),
                    "frac": (v.get("roofline") or {}).get("frac")}
    st = out.get("symbolic_tx")
    if st:
        f["symbolic_tx_wall_s"] = {n.replace(".sol.o", ""): c.get("wall_s") for n, c in st.get("contracts", {}).items()}
    ma = out.get("myth_analyze")
    if ma:
        m = {"contracts": ma.get("contracts_analysed"), "job_wall_s": ma.get("job_wall_s"),
             "host_fraction": ma.get("host_fraction"), "totals": ma.get("totals")}
        cpu = ma.get("cpu_baseline")
        if cpu:
            m["cpu"] = _pick(cpu, ("value", "wall_s", "cores", "issue_sets_match", "counters_match",
                                   "unknown_confirmations"))
            m["mismatched"] = (cpu.get("mismatched") or [])[:4]
        for k in ("solver", "c3"):
            if k in ma:
                m[k] = ma[k]
        f["myth_analyze"] = m
    if out.get("c3_bectoken"):
        f["c3_bectoken"] = out["c3_bectoken"].get("summary", out["c3_bectoken"])
    line["fields"] = f
    line["full_record"] = full_record
    line = _r(line)
    # the limit is the contract: shed the least important summaries first
    for k in ("symbolic_tx_wall_s", "taint_lanes", "c2_large_contract", "c2_unbucketed", "taint_c2",
              "hooked_c2", "c3_bectoken", "myth_analyze"):
        if len(json.dumps(line)) <= LINE_LIMIT:
            break
        line["fields"].pop(k, None)
    if len(json.dumps(line)) > LINE_LIMIT and line.get("cpu_baseline"):
        line["cpu_baseline"]["sample"] = line["cpu_baseline"].get("sample", "")[:120]
    return line


# the opcodes the default detection modules hook (union of
# analysis/module/modules/*.py pre_hooks / post_hooks; pruner plugins add more)
DEFAULT_MODULE_PRE = ["ADD", "MUL", "EXP", "SUB", "SSTORE", "SLOAD", "JUMP", "JUMPI", "STOP",
                      "RETURN", "REVERT", "INVALID", "CALL", "CALLCODE", "DELEGATECALL", "STATICCALL",
                      "CREATE", "CREATE2", "SELFDESTRUCT", "BLOCKHASH", "LOG1", "MSTORE"]
DEFAULT_MODULE_POST = ["ORIGIN", "BLOCKHASH", "COINBASE", "GASLIMIT", "TIMESTAMP", "NUMBER", "CALL",
                       "STATICCALL", "DELEGATECALL", "CALLCODE"]


def run_hooked_c2(dev, n_lanes, rank):
    """C2's lanes through the batched LaserEVM (host mirror, BFS) with a counting
    hook on every opcode the default detection modules hook: how `myth analyze`
    drives kernel 1.  Every hooked instruction yields the lane to the host,
    which fires the hooks in the reference's order and resumes it.  Reports
    lane-steps/s, hook events/s and the wall time split into device (kernel-1
    launches) and host."""
    from mythril_amd import workloads
    from mythril_amd.laser import Account, Disassembly, LaserEVM, MessageCallTransaction, WorldState
    from mythril_amd.laser.strategy import BreadthFirstSearchStrategy
    from mythril_amd.laser.transaction import _setup_global_state_for_execution
    from mythril_amd.lanes import limbs_to_word

    code = workloads.bytecode("overflow.sol.o")
    b = workloads.c2_batch(n_lanes, seed=workloads.C2_SEED + 7 + rank)
    laser = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy, execution_timeout=0)
    events = [0]

    def hook(_state):
        events[0] += 1
    laser.register_hooks("pre", {op: [hook] for op in DEFAULT_MODULE_PRE})
    laser.register_hooks("post", {op: [hook] for op in DEFAULT_MODULE_POST})
    dis = Disassembly(code)
    for i in range(n_lanes):
        ws = WorldState()
        acct = Account(workloads.CONTRACT, code=dis, concrete_storage=True)
        for k in range(int(b.storage_count[i])):
            acct.storage.printable_storage[limbs_to_word(b.storage[i, k, :8])] = \
                limbs_to_word(b.storage[i, k, 8:])
        ws.put_account(acct)
        tx = MessageCallTransaction(world_state=ws, callee_account=acct, caller=workloads.ATTACKER,
                                    call_data=bytes(b.calldata[i, :int(b.calldata_len[i])]),
                                    gas_price=1, gas_limit=8_000_000, origin=workloads.ATTACKER,
                                    code=dis, call_value=0)
        _setup_global_state_for_execution(laser, tx)
    t0 = time.perf_counter()
    laser.exec()
    wall = time.perf_counter() - t0
    dev_s = laser.device_ms / 1e3
    return {"metric": "lane-steps/s with the default modules' hooks (kernel 1 + host LaserEVM)",
            "lanes": n_lanes, "lane_steps": int(laser.lane_steps), "hook_events": events[0],
            "launches": int(laser.launches), "wall_s": wall, "device_s": dev_s,
            "host_s": wall - dev_s, "lane_steps_per_s": laser.lane_steps / wall,
            "hook_events_per_s": events[0] / wall,
            "hooked_opcodes": {"pre": DEFAULT_MODULE_PRE, "post": DEFAULT_MODULE_POST}}


def _c2_laser_states(laser, n_lanes, seed):
    from mythril_amd import workloads
    from mythril_amd.laser import Account, Disassembly, MessageCallTransaction, WorldState
    from mythril_amd.laser.transaction import _setup_global_state_for_execution
    from mythril_amd.lanes import limbs_to_word
    b = workloads.c2_batch(n_lanes, seed=seed)
    dis = Disassembly(workloads.bytecode("overflow.sol.o"))
    for i in range(n_lanes):
        ws = WorldState()
        acct = Account(workloads.CONTRACT, code=dis, concrete_storage=True)
        for k in range(int(b.storage_count[i])):
            acct.storage.printable_storage[limbs_to_word(b.storage[i, k, :8])] = \
                limbs_to_word(b.storage[i, k, 8:])
        ws.put_account(acct)
        tx = MessageCallTransaction(world_state=ws, callee_account=acct, caller=workloads.ATTACKER,
                                    call_data=bytes(b.calldata[i, :int(b.calldata_len[i])]),
                                    gas_price=1, gas_limit=8_000_000, origin=workloads.ATTACKER,
                                    code=dis, call_value=0)
        _setup_global_state_for_execution(laser, tx)


def run_taint_c2(dev, n_lanes, rank, modes=("device", "host")):
    """Taint lanes in situ: C2's lanes through the batched
    LaserEVM (BFS) with the integer and TxOrigin detection modules registered
    (their hook logic restated in tests/refmodules.py: the reference's modules
    cannot be imported here) plus ArbitraryStorage, ArbitraryJump, UserAssertions,
    Exceptions and StateChangeAfterCall.  `device`: their batch-safe hooks run
    as k_sym_step actions and record replays (laser/taint.py); `host`: the same
    hooks as host events.  Same annotations, state annotations and issues
    either way (tests/test_gpu_taint.py)."""
    sys.path.insert(0, str(Path(__file__).resolve().parent / "tests"))
    import refmodules
    from refmodules import hooks_of
    names = ("IntegerArithmetics", "TxOrigin", "ArbitraryStorage", "ArbitraryJump", "UserAssertions",
             "Exceptions", "StateChangeAfterCall")
    from mythril_amd.laser import LaserEVM
    from mythril_amd.laser import taint as tnt
    from mythril_amd.laser.strategy import BreadthFirstSearchStrategy
    out = {"metric": "lane-steps/s with seven default detection modules (kernel 1 taint lanes + host LaserEVM)",
           "lanes": n_lanes, "modules": list(names),
           "modules_source": "tests/refmodules.py (restated: the reference's modules need z3)"}
    saved = tnt.BATCH_SAFE
    try:
        for mode in modes:
            tnt.BATCH_SAFE = saved if mode == "device" else {}
            laser = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy, execution_timeout=0)
            laser.track_objects = True
            mods = [getattr(refmodules, m)() for m in names]
            laser.register_hooks("pre", hooks_of(mods, "pre"))
            laser.register_hooks("post", hooks_of(mods, "post"))
            _c2_laser_states(laser, n_lanes, workloads_seed(rank))
            t0 = time.perf_counter()
            laser.exec()
            wall = time.perf_counter() - t0
            dev_s = laser.device_ms / 1e3
            out[mode] = {"lane_steps": int(laser.lane_steps), "launches": int(laser.launches),
                         "wall_s": wall, "device_s": dev_s, "host_s": wall - dev_s,
                         "lane_steps_per_s": laser.lane_steps / wall,
                         "issues": sum(len(m.issues) for m in mods)}
    finally:
        tnt.BATCH_SAFE = saved
    if "device" in out and "host" in out:
        out["speedup"] = out["device"]["lane_steps_per_s"] / out["host"]["lane_steps_per_s"]
    return out


def workloads_seed(rank):
    from mythril_amd import workloads
    return workloads.C2_SEED + 11 + rank


def run_two_streams(dev, batch, code, steps, local, barrier):
    """The same 65,536-lane C2 batch on a second library context (its own HIP
    stream and lane buffers) while the first runs it too: K batches per stream,
    issued from two host threads (ctypes drops the GIL inside mg_run_batches).
    A block owns its CU's LDS, so the second stream's blocks start on the CUs
    the first batch's short waves free while its slowest waves (the sendeth
    path) still run: the tail of one batch is filled by the next.  Reported
    beside `value`, never as it (`value` keeps one batch in flight)."""
    import threading
    from mythril_amd import workloads
    from mythril_amd.device import GpuDevice
    dev2 = GpuDevice(local)
    try:
        cid2 = dev2.load_code(code)
        b2 = workloads.slim_copy(batch)
        if cid2 != int(batch.code_id[0]):
            b2.code_id[:] = cid2
        dev2.alloc(batch.shape, coverage=True)
        dev2.upload(b2)
        # warm up at the timed batch count: a larger statistics buffer is re-allocated
        # on first use, and hipFree waits for the whole device (both streams)
        dev.run_batches(steps)
        dev2.run_batches(steps)
        res = [None, None]

        def go(k, d):
            res[k] = d.run_batches(steps)
        barrier()
        t0 = time.perf_counter()
        th = [threading.Thread(target=go, args=(k, d)) for k, d in enumerate((dev, dev2))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        barrier()
        el = time.perf_counter() - t0
        lane_steps = sum(st.lane_steps for r in res for st in r)
        if any(st.running for r in res for st in r):
            raise RuntimeError("a two-stream C2 batch ended with lanes still running")
        per = [sum(st.lane_steps for st in r) for r in res]
        return {"value": lane_steps / el, "unit": "lane-steps/s", "streams": 2, "batches_per_stream": steps,
                "lanes_per_batch": batch.n, "ms_per_batch": 1000.0 * el / (2 * steps),
                "lane_steps_per_stream": per,
                "kernel_ms_per_batch": float(np.mean([st.kernel_ms for r in res for st in r]))}
    finally:
        dev2.close()


def run_large(dev, args, rank, barrier):
    """C2's lane generator on the reference's 3,523-instruction disassembler
    fixture (workloads.large_code: 16 selectors, bucketed): the pre-decoded
    code fills LDS with the push immediates left in HBM (parity:
    tests/test_gpu_lds_plan.py::test_large_code_staged_prefix_with_runs)."""
    from mythril_amd import dist as mdist, workloads
    from mythril_amd.lanes import bucket_order, permuted
    code = workloads.large_code()
    cid = dev.load_code(code)
    b = workloads.c2_batch(args.lanes, code_id=cid, seed=workloads.C2_SEED + 0x100 + rank,
                           stack_cap=1024, mem_cap=4096, rec_cap=args.rec_cap,
                           selectors=workloads.dispatch_selectors(code))
    b = permuted(b, bucket_order(b))
    dev.alloc(b.shape, coverage=True)
    dev.upload(workloads.slim_copy(b))
    dev.run_batches(2)
    barrier()
    t0 = time.perf_counter()
    st = dev.run_batches(args.large_steps)
    barrier()
    el = time.perf_counter() - t0
    el, steps = mdist.reduce_timing(el, float(sum(s.lane_steps for s in st)))
    return {"value": steps / el, "unit": "lane-steps/s", "instructions": dev.n_instr(cid),
            "lanes_per_gpu": args.lanes,
            "ms_per_step": 1000.0 * el / args.large_steps,
            "kernel_ms_per_batch": float(np.mean([s.kernel_ms for s in st])),
            "escaped_lanes_per_batch": float(np.mean([s.escaped for s in st])),
            "code": "tests/golden/disassembly.json (disassembler_test.py:8-10)"}


SYMBOLIC_TX_CODES = ("overflow.sol.o", "exceptions.sol.o", "flag_array.sol.o")


def symbolic_lane_batch(dev, lanes: int, order: str = "code"):
    """`lanes` symbolic lanes: the initial state of a symbolic message call
    (transaction/symbolic.py:105-150: symbolic calldata, sender, value, gas
    price; symbolic storage, as `myth analyze -f` analyses a runtime code) into
    each of the reference's precompiled contracts.  order "code": contiguous
    runs of one contract (a wave's lanes share their code, so their stack
    depths, arena sizes and memory offsets line up and the planes' writes
    coalesce); "rr": dealt round-robin.  Returns (LaserEVM, batch)."""
    from dataclasses import replace
    from mythril_amd import workloads
    from mythril_amd.lanes import _ALL_FIELDS, _SYM_FIELDS, LaneBatch, LaneShape
    from mythril_amd.laser import (Account, BreadthFirstSearchStrategy, Disassembly, LaserEVM,
                                   MessageCallTransaction, SymbolicCalldata, WorldState)
    from mythril_amd.laser.transaction import ACTORS
    from mythril_amd.smt.expr import Or, symbol_factory
    codes = json.loads((ROOT / "tests" / "golden" / "bytecodes.json").read_text())
    laser = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy, execution_timeout=0)
    states = []
    for k, name in enumerate(sorted(codes)):
        ws = WorldState()
        ws.put_account(Account(ACTORS["CREATOR"]))
        acct = Account(workloads.CONTRACT, code=Disassembly(workloads.bytecode(name)), concrete_storage=False)
        ws.put_account(acct)
        txid = str(k + 1)
        sender = symbol_factory.BitVecSym(f"sender_{txid}", 256)
        tx = MessageCallTransaction(world_state=ws, identifier=txid,
                                    gas_price=symbol_factory.BitVecSym(f"gas_price{txid}", 256),
                                    gas_limit=8_000_000, origin=sender, caller=sender, callee_account=acct,
                                    call_data=SymbolicCalldata(txid),
                                    call_value=symbol_factory.BitVecSym(f"call_value{txid}", 256))
        gs = tx.initial_global_state()
        gs.transaction_stack.append((tx, None))
        gs.world_state.constraints.append(
            Or(*[tx.caller == symbol_factory.BitVecVal(a, 256) for a in ACTORS.values()]))
        states.append(gs)
    shape = laser._shape(states)
    # 65,536 lanes: a 128-word stack and 1 KiB of memory per lane keep the
    # planes (memory byte tags included) within a few hundred MB
    shape = replace(shape, stack_cap=128, mem_cap=1024, storage_cap=64, rec_cap=512)
    small = LaneBatch(shape)
    for i, gs in enumerate(states):
        laser._pack(small, i, gs)
    big = LaneBatch(replace(shape, n=lanes))
    idx = (np.arange(lanes) * len(states) // lanes) if order == "code" else np.arange(lanes) % len(states)
    for f in _ALL_FIELDS + _SYM_FIELDS:
        src = getattr(small, f, None)
        if src is not None:
            getattr(big, f)[...] = src[idx]
    return laser, big


def run_symbolic_lanes(dev, lanes: int, reps: int = 5, profile: bool = True, order: str = "code"):
    """k_sym_step at `lanes` lanes: every lane runs from the
    start of its symbolic message call to its first stop -- MG_FORK at a
    symbolic JUMPI (the dispatcher's selector compare), an escape or a halt --
    in one launch.  Timed per launch with the device's HIP events (the events
    bracket kernel 1's no-op pass over the symbolic lanes too: k_lane_step
    leaves them to k_sym_step); the image is re-uploaded before each launch,
    outside the timed region.  The roofline prices the opcode histogram a
    profiling pass of k_sym_step counts (mg_step_profile) with §8(d)'s table,
    plus 4 bytes of tag per stack word moved and 16 bytes per arena node
    created."""
    from mythril_amd import roofline
    from mythril_amd.lanes import MG_FORK, STATUS_NAMES, LaneBatch
    laser, b = symbolic_lane_batch(dev, lanes, order)
    n0 = int(b.n_nodes.sum())
    dev.alloc(b.shape)
    dev.upload(b)
    dev.step()
    ms, steps = [], 0
    for _ in range(reps):
        dev.upload(b)
        st = dev.step()
        ms.append(st.kernel_ms)
        steps = st.lane_steps
    out_b = LaneBatch(b.shape)
    dev.download(out_b)
    created = int(out_b.n_nodes.sum()) - n0
    statuses = {STATUS_NAMES.get(int(k), str(int(k))): int(v)
                for k, v in zip(*np.unique(out_b.status, return_counts=True))}
    if not profile:            # the timed launches alone (PMC passes of k_sym_step)
        if os.environ.get("MG_SYM_MAXSTEPS"):
            # diagnostic: every lane stops after K steps (the write traffic's slope per step)
            k = int(os.environ["MG_SYM_MAXSTEPS"])
            ms = []
            for _ in range(reps):
                dev.upload(b)
                st = dev.step(max_steps=k)
                ms.append(st.kernel_ms)
                steps = st.lane_steps
        if os.environ.get("MG_SYM_FLUSH"):
            # diagnostic: a kernel-2 launch that streams ~1 GB between the upload and
            # each launch, so the upload's dirty lines leave L2 / MALL before the
            # kernel runs instead of during it (scripts/r05/gpu_symflush.sh)
            from mythril_amd.smt import synth
            fprog, fmodels = synth.c4_batch(1_000_000, 4096)
            dev.eval_upload(fprog, fmodels)
            ms = []
            for _ in range(reps):
                dev.upload(b)
                dev.eval_run()
                st = dev.step()
                ms.append(st.kernel_ms)
        kms = float(np.median(ms))
        return {"lanes": lanes, "lane_steps_per_launch": int(steps), "kernel_ms": kms, "kernel_ms_all": ms,
                "lane_steps_per_s": steps / (kms / 1e3), "statuses": statuses}
    dev.upload(b)
    op_counts, extra = dev.step_profile()
    ops, byts, psteps = roofline.algorithmic_work(op_counts, extra)
    words = float((op_counts.astype(np.float64) * roofline.WORDS).sum())
    byts += 4.0 * words + 16.0 * created
    kms = float(np.median(ms))
    sec = kms / 1e3
    gbs, tops = byts / sec / 1e9, ops / sec / 1e12
    hbm = gbs / roofline.HBM_PEAK_GBS >= tops / roofline.VALU_PEAK_TOPS
    roof = roofline.with_sustained({
        "bound": "hbm" if hbm else "valu-int32",
        "achieved": gbs if hbm else tops,
        "peak": roofline.HBM_PEAK_GBS if hbm else roofline.VALU_PEAK_TOPS,
        "unit": "GB/s" if hbm else "T int32-ops/s",
        "frac": gbs / roofline.HBM_PEAK_GBS if hbm else tops / roofline.VALU_PEAK_TOPS,
        "traffic": roofline.pmc_traffic("k_sym_step")[0],
        "kernel": "k_sym_step", "kernel_ms": kms,
        "algorithmic_bytes_per_launch": byts, "algorithmic_int32_ops_per_launch": ops,
        "bytes_per_lane_step": byts / max(psteps, 1.0), "int32_ops_per_lane_step": ops / max(psteps, 1.0),
        "arena_nodes_created": created,
    })
    return {"metric": "symbolic lane-steps/s (k_sym_step)", "lanes": lanes, "codes": int(len(set(b.code_id.tolist()))),
            "lane_steps_per_launch": int(steps), "kernel_ms": kms, "kernel_ms_all": ms,
            "lane_steps_per_s": steps / sec, "forked": int((out_b.status == MG_FORK).sum()),
            "statuses": statuses, "roofline": roof,
            "workload": "symbolic message call into each of the 18 precompiled reference contracts "
                        "(symbolic calldata/sender/value, symbolic storage), dealt round-robin; "
                        "each lane runs to its first fork, escape or halt"}


def run_taint_lanes(dev, lanes: int, rank: int = 0, reps: int = 5, order: str = "code", profile: bool = True):
    """k_sym_step at `lanes` taint lanes, the kernel alone: the
    first launch of `taint_c2`'s batch -- C2's lanes with the seven modules'
    batch-safe hooks as device actions -- packed by the batched LaserEVM for
    4,096 distinct C2 calls and dealt round-robin to `lanes` lanes, then run to
    the first host event (a non-batch-safe hook, a halt, an escape) in one
    launch.  The host replay of the records (what `taint_c2` adds on top) is
    not part of this figure."""
    from dataclasses import replace
    sys.path.insert(0, str(Path(__file__).resolve().parent / "tests"))
    import refmodules
    from refmodules import hooks_of
    from mythril_amd.lanes import _ALL_FIELDS, _TAINT_FIELDS, LaneBatch, MG_RUNNING, STATUS_NAMES
    from mythril_amd.laser import LaserEVM
    from mythril_amd.laser import svm as svm_mod
    from mythril_amd.laser import taint as tnt
    from mythril_amd.laser.strategy import BreadthFirstSearchStrategy
    names = ("IntegerArithmetics", "TxOrigin", "ArbitraryStorage", "ArbitraryJump", "UserAssertions",
             "Exceptions", "StateChangeAfterCall")
    laser = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy, execution_timeout=0)
    laser.track_objects = True
    mods = [getattr(refmodules, m)() for m in names]
    laser.register_hooks("pre", hooks_of(mods, "pre"))
    laser.register_hooks("post", hooks_of(mods, "post"))
    distinct = min(4096, lanes)
    _c2_laser_states(laser, distinct, workloads_seed(rank))
    states = laser.work_list[:]
    plan = tnt.TaintPlan(laser)
    laser._plan = plan
    laser._tl = [tnt.LaneTaint() for _ in states]
    shape = laser._shape(states, True)
    small = LaneBatch(shape)
    for i, st in enumerate(states):
        laser._pack(small, i, st)
        small.steps[i] = 0
    big = LaneBatch(replace(shape, n=lanes))
    idx = np.arange(lanes) % distinct
    if order == "code":
        # C2's bucketing (code, selector, calldata length; lanes.bucket_order): a
        # wave's lanes walk one function's path, so their writes coalesce
        from mythril_amd.lanes import bucket_order
        idx = idx[bucket_order(_rows(small, idx))]
    for f in _ALL_FIELDS + _TAINT_FIELDS:
        src = getattr(small, f, None)
        if src is not None:
            getattr(big, f)[...] = src[idx]
    mask = svm_mod._mask(laser._hooked_ops())
    dev.alloc(big.shape)
    dev.set_taint_program(plan.actions)
    laser._upload_force(dev)
    ms, steps = [], 0
    for _ in range(reps + 1):
        dev.upload(big)
        st = dev.step(mask)
        ms.append(st.kernel_ms)
        steps = st.lane_steps
    ms = ms[1:]
    out_b = LaneBatch(big.shape)
    dev.download(out_b)
    statuses = {STATUS_NAMES.get(int(k), str(int(k))): int(v)
                for k, v in zip(*np.unique(out_b.status, return_counts=True))}
    kms = float(np.median(ms))
    out = {"metric": "taint lane-steps/s (k_sym_step, device actions; host replay excluded)",
           "lanes": lanes, "distinct_calls": distinct, "modules": list(names),
           "lane_steps_per_launch": int(steps), "kernel_ms": kms, "kernel_ms_all": ms,
           "lane_steps_per_s": steps / (kms / 1e3) if kms else None, "statuses": statuses,
           "running_after": int((out_b.status == MG_RUNNING).sum()), "order": order}
    if profile:
        # §8(d)'s bytes per lane-step from the launch's own opcode histogram (an
        # untimed profiling pass of the same image), plus what a taint lane moves
        # besides: a 4-byte object handle per stack word moved and the hook
        # records it writes (4 bytes a word; MG_REC_ANNOT / MG_REC_HOOK)
        from mythril_amd import roofline
        dev.upload(big)
        op_counts, extra = dev.step_profile(mask)
        ops, byts, psteps = roofline.algorithmic_work(op_counts, extra)
        words = float((op_counts.astype(np.float64) * roofline.WORDS).sum())
        rec_bytes = 4.0 * float(out_b.rec_len.astype(np.float64).sum())
        byts += 4.0 * words + rec_bytes
        traffic, src = roofline.pmc_traffic("k_sym_step_taint")
        sec = kms / 1e3
        gbs = byts / sec / 1e9
        out["roofline"] = roofline.with_sustained({
            "bound": "hbm", "achieved": gbs, "peak": roofline.HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / roofline.HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
            "kernel": "k_sym_step (taint lanes)", "kernel_ms": kms,
            "algorithmic_bytes_per_launch": byts, "algorithmic_int32_ops_per_launch": ops,
            "record_bytes_per_launch": rec_bytes, "bytes_per_lane_step": byts / max(psteps, 1.0),
            "traffic_over_algorithmic": (traffic / byts) if traffic else None})
    return out


def run_symbolic_tx(dev, replicas: int, tx_count: int, n_seeds: int, escape_handler=None, log=None):
    """C3 in situ (BASELINE configs[2] needs solc for BECToken; the reference's
    own precompiled contracts stand in): `-t tx_count` symbolic transactions
    (svm.py:214-275, transaction/symbolic.py:105-150) through the batched
    LaserEVM with the fork filter ON (svm.py:319-326) and the per-transaction
    reachability filter (svm.py:244-249).  Symbolic lanes run on kernel 1
    (store chains, symbolic memory, symbolic SHA3); every fork filter group and
    reachability round is one kernel-2 launch over the model cache plus
    `n_seeds` witness seeds (laser/witness.py).  A query no candidate satisfies
    goes to the exact procedure (smt/exact.py), and its fork is pruned on unsat
    or on a budget timeout, as is_possible prunes (constraints.py:33-43);
    escaped paths (no host handler) are dropped and counted.  Runtime codes are analysed as `myth analyze -f` does (symbolic
    storage); flag_array is deployed concretely first.  `replicas` copies of the
    deployed world state run together (one contract per replica, independent
    paths) for a batch that fills the GPU; replicas=1 is one analysis.  With
    N ranks, replicas x N copies are dealt over the ranks and the open states
    are rebalanced at every transaction boundary (laser/sharded.py
    execute_symbolic_transactions): per-GPU work is fixed (weak scaling); the
    whole-job rates sum the ranks' work over the slowest rank's wall time."""
    from copy import copy
    from mythril_amd import workloads
    from mythril_amd.laser import (Account, BreadthFirstSearchStrategy, Disassembly, LaserEVM, WorldState,
                                   execute_contract_creation)
    from mythril_amd import dist as mdist
    from mythril_amd.laser.sharded import execute_symbolic_transactions
    from mythril_amd.laser.transaction import ACTORS, tx_id_manager
    from mythril_amd.laser.witness import WitnessSeeds
    from mythril_amd.smt import solver
    from mythril_amd.smt.keccak_manager import keccak_function_manager
    creator = ACTORS["CREATOR"]
    out = {"metric": "in-situ constraint-evals/s of the fork and reachability filters (kernel 2) "
                     "+ symbolic lane-steps/s (kernel 1)",
           "mode": "kernel-2 prefilter (LRU + witness seeds), then the exact procedure "
                   "(mythril_amd/smt/exact.py: bit-blasting + CDCL) on what it leaves open: forks "
                   "pruned on unsat and on a budget timeout as is_possible does; escapes stepped by "
                   "the handler given (bench: tests/symref.py), else dropped (counted)",
           "transactions": tx_count, "replicas_per_gpu": replicas, "seed_models": n_seeds, "contracts": {}}
    from mythril_amd.smt.exact import ExactSolver
    from mythril_amd.smt.search import SatSearchBackend
    saved_cache, saved_backend = solver.model_cache, solver.solver_backend
    try:
        for name in SYMBOLIC_TX_CODES:
            gc.collect()                     # the earlier fields' garbage is not this field's work
            keccak_function_manager.reset()
            tx_id_manager.restart_counter()
            solver.get_model.cache_clear()
            code = workloads.bytecode(name)
            ws = WorldState()
            ws.put_account(Account(creator))
            if name == "flag_array.sol.o":
                laser = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy, execution_timeout=0)
                laser.open_states = [ws]
                execute_contract_creation(laser, None, creator, creator, code, 8_000_000, 1, 10 ** 17)
                if len(laser.open_states) != 1:
                    out["contracts"][name] = {"error": "deployment did not complete"}
                    continue
                ws = laser.open_states[0]
                addr = next(a for a in ws.accounts if a != creator)
            else:
                addr = workloads.CONTRACT
                ws.put_account(Account(addr, code=Disassembly(code), concrete_storage=False))
            mc = solver.ModelCache(device=dev)
            seeds = WitnessSeeds([code], n=n_seeds, storage_names=[f"Storage{addr}"], balance_names=["balance"])
            mc.seed_source = seeds
            solver.model_cache = mc
            backend = SatSearchBackend(mc, search=False, exact=ExactSolver(), exact_ms=60000)
            solver.set_solver_backend(backend)
            laser = LaserEVM(requires_statespace=False, device=dev, strategy=BreadthFirstSearchStrategy, execution_timeout=0,
                             transaction_count=tx_count, escape_handler=escape_handler)
            if log:
                log(f"symbolic_tx {name}")
                laser.register_laser_hooks("start_sym_trans", lambda: log(
                    f"symbolic_tx {name}: transaction with {len(laser.open_states)} open states"))
            ends = {"return_or_stop": 0, "revert": 0}
            laser.register_laser_hooks("transaction_end", lambda s, tx, r, revert: ends.__setitem__(
                "revert" if revert else "return_or_stop", ends["revert" if revert else "return_or_stop"] + 1))
            rank, world = mdist.rank_world()
            laser.open_states = [copy(ws) for _ in range(replicas * world)]
            t0 = time.perf_counter()
            execute_symbolic_transactions(laser, addr)
            wall = time.perf_counter() - t0
            job_wall, job_steps = mdist.reduce_timing(wall, float(laser.lane_steps))
            _, job_evals = mdist.reduce_timing(wall, float(mc.device_evals))
            k1_s, k2_s = laser.device_ms / 1e3, mc.device_ms / 1e3
            st = mc.stats
            answered = st["lru_hits"] + st["seed_hits"]
            out["contracts"][name] = {
                "wall_s": wall, "kernel1_s": k1_s, "kernel2_s": k2_s, "host_s": wall - k1_s - k2_s,
                "lane_steps": int(laser.lane_steps), "lane_steps_per_s": laser.lane_steps / wall,
                "launches_kernel1": int(laser.launches), "forks": laser.forks,
                "tx_ends": ends, "open_states": len(laser.open_states),
                "escapes_dropped": laser.escapes_dropped,
                "fork_filter": dict(laser.fork_stats),
                "queries": st["queries"], "lru_hits": st["lru_hits"], "seed_hits": st["seed_hits"],
                "unknown": st["misses"],
                "prefilter_hit_rate": answered / st["queries"] if st["queries"] else None,
                "constraint_evals": int(mc.device_evals), "launches_kernel2": int(mc.launches),
                "constraint_evals_per_s_kernel": mc.device_evals / k2_s if k2_s else None,
                "constraint_evals_per_s_wall": mc.device_evals / wall,
                "keccak_symbolic_inputs": sum(len(v) for v in keccak_function_manager.symbolic_inputs.values()),
                "exact": {k: backend.stats[k] for k in ("exact_sat", "exact_unsat", "exact_timeout")},
                "exact_ms": backend.exact.stats["ms"],
                "ranks": world, "job_lane_steps_per_s": job_steps / job_wall,
                "job_constraint_evals_per_s_wall": job_evals / job_wall,
            }
    finally:
        solver.model_cache = saved_cache
        solver.set_solver_backend(saved_backend)
        keccak_function_manager.reset()
        tx_id_manager.restart_counter()
        solver.get_model.cache_clear()
    return out


def _myth_analyze_rows(device, k2, tx_count: int, names, log=None):
    """tests/analyze.py over `names`: per contract the issue table, the
    confirmations (sat / unsat / timeout / unknown), escapes dropped, wall / kernel time and the
    in-situ rates."""
    import analyze
    rows = {}
    for name in names:
        gc.collect()
        if log:
            log(f"myth_analyze: {name}")
        issues, info = analyze.analyze(name, None, tx_count, device, k2)
        k1_s = info["device_ms"] / 1e3
        k2_s = info["k2_ms"] / 1e3
        rows[name] = {"issues": [list(r) for r in analyze.issue_table(issues)],
                      "confirmations": info["confirmations"], "escapes_dropped": info["escapes_dropped"],
                      "wall_s": info["wall_s"], "kernel1_s": k1_s, "kernel2_s": k2_s,
                      "lane_steps": int(info["lane_steps"]), "constraint_evals": int(info["device_evals"]),
                      "launches_kernel2": int(info["kernel2_launches"]), "forks": info["forks"],
                      "fork_filter": {k: info["fork_filter"].get(k) for k in ("groups", "queries", "kept", "pruned",
                                                                               "unknown")},
                      "search": {k: info["search"][k] for k in ("calls", "refuted", "seed", "search", "unknown",
                                                                "exact_sat", "exact_unsat", "exact_timeout")
                                 if k in info["search"]},
                      "exact_ms": (info.get("exact") or {}).get("ms", 0),
                      "constraint_evals_per_s_wall": info["device_evals"] / info["wall_s"] if info["wall_s"] else None}
    return rows


def _rows(batch, idx):
    """A view of `batch` with lanes idx (only the fields bucket_order reads)."""
    class _V:
        pass
    v = _V()
    v.code_id, v.calldata, v.calldata_len = batch.code_id[idx], batch.calldata[idx], batch.calldata_len[idx]
    v.shape, v.n = batch.shape, len(idx)
    return v


def run_myth_analyze(dev, tx_count: int, log=None, names=None, cpu: bool = True):
    """C3-shaped (BECToken needs solc, the reference's 18
    precompiled test contracts stand in): ``myth analyze -f <code> -t tx_count``
    with every detection module, as tests/analyze.py runs the reference's
    integration rows -- symbolic creation then tx_count symbolic message calls,
    BFS + BoundedLoopsStrategy(3), max depth 128, the mutation pruner, the
    modules' hooks (tests/refmodules.py, restated: the reference's modules need
    z3), the fork and reachability filters and every issue confirmation on
    kernel 2 (model cache, witness seeds, guided search and the keccak-axiom
    refutations, then the exact procedure of smt/exact.py on what they leave
    open: unsat and budget timeouts drop the issue and prune the fork, as the
    reference does), escapes stepped by the tests/symref.py handler so no path
    is dropped.  Contracts are dealt round-robin over the ranks (total work
    fixed).  The CPU comparator runs the same harness on rank 0 with the C
    oracles as kernels 1 and 2 (oracle/evm_ref.c single-threaded,
    oracle/bv_ref.c on the host's CPU share) and reports whether the issue
    sets agree."""
    sys.path.insert(0, str(Path(__file__).resolve().parent / "tests"))
    import tempfile
    import fnames
    from mythril_amd import dist as mdist
    from mythril_amd import workloads
    from mythril_amd.laser.disassembly import SignatureDB
    rank, world = mdist.rank_world()
    names = sorted(names or workloads.bytecode_names())
    saved_dir = os.environ.get("MYTHRIL_DIR")
    with tempfile.TemporaryDirectory() as sigdir:
        # the signature database the reference builds by importing the inputs'
        # sources (function names of the issues)
        fnames.signature_db(Path(sigdir))
        os.environ["MYTHRIL_DIR"] = sigdir
        SignatureDB._reset()
        try:
            rows = _myth_analyze_rows(dev, dev, tx_count, names[rank::world], log)
            cpu_rows = None
            if cpu and rank == 0 and world == 1:
                from oracle_device import OracleDevice, OracleK2
                cpu_rows = _myth_analyze_rows(OracleDevice(), OracleK2(), tx_count, names, log)
        finally:
            if saved_dir is None:
                os.environ.pop("MYTHRIL_DIR", None)
            else:
                os.environ["MYTHRIL_DIR"] = saved_dir
            SignatureDB._reset()
    tot = {k: sum(r[k] for r in rows.values()) for k in ("wall_s", "kernel1_s", "kernel2_s", "lane_steps",
                                                         "constraint_evals", "escapes_dropped")}
    tot["issues"] = sum(len(r["issues"]) for r in rows.values())
    tot["unknown_confirmations"] = sum(r["confirmations"]["unknown"] for r in rows.values())
    tot["unsat_confirmations"] = sum(r["confirmations"].get("unsat", 0) for r in rows.values())
    tot["timeout_confirmations"] = sum(r["confirmations"].get("timeout", 0) for r in rows.values())
    for k in ("exact_sat", "exact_unsat", "exact_timeout"):
        tot[k] = sum(r["search"].get(k, 0) for r in rows.values())
    tot["exact_s"] = sum(r.get("exact_ms", 0) for r in rows.values()) / 1e3
    tot["forks_pruned"] = sum(r["fork_filter"].get("pruned", 0) for r in rows.values())
    tot["forks_unknown"] = sum(r["fork_filter"].get("unknown", 0) for r in rows.values())
    job_wall, job_evals = mdist.reduce_timing(tot["wall_s"], float(tot["constraint_evals"]))
    out = {"metric": "myth analyze -f <code> -t %d, all detection modules, over the 18 reference "
                     "contracts: contracts/s and in-situ constraint-evals/s" % tx_count,
           "mode": "modules on; queries on kernel 2 (quick-sat, witness seeds, guided search), the rest "
                   "decided by the exact procedure (mythril_amd/smt/exact.py): unsat and budget timeouts "
                   "prune / refute as the reference's z3 does; escapes stepped by the tests/symref.py handler",
           "transactions": tx_count, "contracts_analysed": len(rows), "ranks": world, "totals": tot,
           "job_wall_s": job_wall, "contracts_per_s": len(names) / job_wall if job_wall else None,
           "job_constraint_evals_per_s_wall": job_evals / job_wall if job_wall else None,
           "host_fraction": 1.0 - (tot["kernel1_s"] + tot["kernel2_s"]) / tot["wall_s"] if tot["wall_s"] else None,
           "contracts": rows}
    if cpu_rows is not None:
        import platform
        from oracle.cpu_baseline import _cores_info, _cpu_share
        cw = sum(r["wall_s"] for r in cpu_rows.values())
        mismatched = sorted(n for n in rows if rows[n]["issues"] != cpu_rows[n]["issues"])
        counters = ("confirmations", "forks", "fork_filter", "search", "escapes_dropped")
        mismatched_counters = sorted(n for n in rows if any(rows[n][k] != cpu_rows[n][k] for k in counters))
        out["cpu_baseline"] = {
            "value": len(cpu_rows) / cw, "unit": "contracts/s", "wall_s": cw,
            **_cores_info(_cpu_share()), "kind": "port",
            "sample": "the same 18 analyses, host layer + oracle/evm_ref.c (1 thread) as kernel 1 + "
                      "oracle/bv_ref.c (%d threads) as kernel 2 (%s)" % (_cpu_share(),
                                                                         _cpu_model() or platform.processor()),
            "issue_sets_match": not mismatched, "mismatched": mismatched,
            "counters_match": not mismatched_counters, "mismatched_counters": mismatched_counters,
            "wall_s_per_contract": {n: r["wall_s"] for n, r in cpu_rows.items()},
            "unknown_confirmations": sum(r["confirmations"]["unknown"] for r in cpu_rows.values())}
        out["speedup_vs_cpu"] = cw / tot["wall_s"] if tot["wall_s"] else None
    return out


def run_c3_bectoken(dev, tx_count: int, log=None):
    """C3 (BASELINE configs[2]): ``myth analyze BECToken.sol -t
    tx_count`` with every detection module on kernels 1 and 2 and the exact
    procedure behind them.  BECToken needs solc 0.4 (absent): tests/bectoken.py
    assembles the contract from its source.  Reports the issue table, whether
    SWC-101 sits at batchTransfer's ``uint256(cnt) * _value`` (CVE-2018-10299),
    the kernel-2 prefilter's hit rate over the queries get_model saw, and the
    exact-procedure calls ("z3 calls") made and avoided."""
    sys.path.insert(0, str(Path(__file__).resolve().parent / "tests"))
    import tempfile
    import analyze
    import bectoken
    import fnames
    from mythril_amd.laser.disassembly import SignatureDB
    saved_dir = os.environ.get("MYTHRIL_DIR")
    with tempfile.TemporaryDirectory() as sigdir:
        fnames.signature_db(Path(sigdir))
        os.environ["MYTHRIL_DIR"] = sigdir
        SignatureDB._reset()
        try:
            if log:
                log(f"C3 BECToken -t {tx_count}")
            gc.collect()
            issues, info = analyze.analyze("BECToken", None, tx_count, dev, dev, code=bectoken.creation(),
                                           search=False)
        finally:
            if saved_dir is None:
                os.environ.pop("MYTHRIL_DIR", None)
            else:
                os.environ["MYTHRIL_DIR"] = saved_dir
            SignatureDB._reset()
    table = [list(r) for r in analyze.issue_table(issues)]
    mul = bectoken.mul_address()
    cache, srch, ex = info["cache"], info["search"], info["exact"] or {}
    answered = cache["lru_hits"] + cache["seed_hits"]
    queries = cache["queries"]
    # every query the kernel-2 prefilter answered, the refutations and the fork
    # filter's quick-sat answers are z3 calls the reference would have made
    exact_calls = srch.get("exact_sat", 0) + srch.get("exact_unsat", 0) + srch.get("exact_timeout", 0)
    summary = {"tx": tx_count, "wall_s": info["wall_s"], "issues": len(table),
               "swc101_at_mul": any(r[0] == "101" and r[1] == mul and r[2] == "batchTransfer(address[],uint256)"
                                    for r in table),
               "prefilter_hit_rate": answered / queries if queries else None,
               "exact_calls": exact_calls, "exact_calls_avoided": answered + srch.get("refuted", 0),
               "exact_s": ex.get("ms", 0) / 1e3, "kernel1_s": info["device_ms"] / 1e3,
               "kernel2_s": info["k2_ms"] / 1e3, "constraint_evals": int(info["device_evals"])}
    return {"metric": "myth analyze BECToken.sol -t %d (C3): issues, prefilter hit rate, exact calls avoided"
                      % tx_count,
            "source": "tests/bectoken.py (assembled from solidity_examples/BECToken.sol; no solc here)",
            "issues": table, "mul_address": mul, "confirmations": info["confirmations"],
            "forks": info["forks"], "fork_filter": info["fork_filter"], "cache": cache,
            "search": srch, "exact": ex, "lane_steps": int(info["lane_steps"]), "summary": summary}


def _cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def run_c4(args, dev, rank, world, barrier, dist_on):
    """C4 (configs[3]): 1M constraint DAGs x 4096 candidate models, DAGs split
    over ranks (strong scaling), models replicated; kernel 2 only in the timed
    region (programs and models resident in HBM)."""
    import torch
    import torch.distributed as dist
    from mythril_amd.smt import synth
    from mythril_amd import dist as mdist
    chunks = synth.c4_chunks(args.c4_dags)
    mine = [c[0] for c in mdist.shard(chunks, rank, world)]
    prog, models = synth.c4_batch(args.c4_dags, args.c4_models, chunks=mine)
    dev.eval_upload(prog, models)
    dev.eval_run()                      # warm-up
    barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.c4_steps):
        kms.append(dev.eval_run())
    barrier()
    el = time.perf_counter() - t0
    fs, sc = dev.eval_download()
    evals = prog.n_dags * models.n_models * args.c4_steps
    n_sat = int((sc > 0).sum())
    el, evals = mdist.reduce_timing(el, float(evals))
    _, n_sat = mdist.reduce_timing(0.0, float(n_sat))
    n_sat = int(n_sat)
    ops, gather_bytes = synth.program_cost(prog)
    ops_nodiv, _ = synth.program_cost(prog, div_cost=0.0)
    div_count = synth.division_count(prog)
    k_ms = float(np.mean(kms))
    ops_launch = ops * models.n_models
    tops = ops_launch / (k_ms / 1e3) / 1e12
    from mythril_amd.roofline import VALU_PEAK_TOPS, pmc_traffic, with_sustained
    traffic, traffic_src = pmc_traffic("k_bv_eval")
    return {
        "metric": "constraint-evals/s (kernel 2, C4: 1M DAGs depth 32 x 4096 models)",
        "value": evals / el, "unit": "constraint-evals/s", "n_gpus": world,
        "ms_per_step": 1000.0 * el / args.c4_steps, "scaling": "strong",
        "config": {"workload": "C4", "dags": args.c4_dags, "models": args.c4_models,
                   "dags_with_a_satisfying_model": n_sat},
        "roofline": _k2_roofline(tops, k_ms, ops_nodiv, models.n_models, {"traffic": traffic,
                     "traffic_unit": "bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_source": traffic_src,
                     "kernel": "k_bv_eval", "kernel_ms": k_ms,
                     "algorithmic_int32_ops_per_launch": ops_launch,
                     "int32_ops_per_eval": ops / max(prog.n_dags, 1),
                     # the §8(d) division charge (32 w^2 per 256-bit div/rem) is most of
                     # `achieved`; without it, and with divisions at the VALU count the
                     # Knuth-D path executes (SQ_INSTS_VALU of the divrem-only class,
                     # profiles/r02/k2_div_valu.json):
                     "without_division_charge": _k2_alt(ops_nodiv, 0.0, models.n_models, k_ms),
                     "division_at_executed_valu": _k2_alt(ops_nodiv, div_count, models.n_models, k_ms,
                                                          executed=True),
                     "divisions_per_eval": div_count / max(prog.n_dags, 1),
                     "model_bytes_per_eval": gather_bytes / max(prog.n_dags, 1)}),
    }


def _k2_roofline(tops_charged, k_ms, ops_nodiv, n_models, extra):
    """C4's roofline.  Headline: the §8(d) int32 ops WITHOUT the
    2,048-op division charge over the INT32 VALU peak -- the charge is not work
    the kernel does (with it the fraction passes the measured sustained peak);
    the charged figure stays beside it.  The measured bound is the
    interpreter's scalar issue (`issue_floor`)."""
    from mythril_amd.roofline import VALU_PEAK_TOPS, k2_issue_floor, sustained_peaks, with_sustained
    tops = ops_nodiv * n_models / (k_ms / 1e3) / 1e12
    floor = k2_issue_floor(k_ms)
    roof = with_sustained({"bound": (floor["bound"] + "-issue") if floor else "valu-int32",
                           "priced_as": "valu-int32",
                           "frac_basis": "§8(d) int32 ops without the division charge / INT32 VALU peak",
                           "achieved": tops, "peak": VALU_PEAK_TOPS, "unit": "T int32-ops/s",
                           "frac": tops / VALU_PEAK_TOPS})
    _, valu_sust = sustained_peaks()
    roof["with_division_charge"] = {"achieved": tops_charged, "frac": tops_charged / VALU_PEAK_TOPS,
                                    "frac_sustained": tops_charged / valu_sust if valu_sust else None}
    if floor:
        roof["issue_floor"] = floor
    roof.update(extra)
    return roof


def _k2_alt(ops_nodiv, div_count, n_models, k_ms, executed=False):
    """Kernel 2's INT32 roofline with another division cost: none, or the
    measured VALU instructions per division (profiles/r02/k2_div_valu.json)."""
    from mythril_amd.roofline import VALU_PEAK_TOPS, division_valu
    per_div = 0.0
    src = None
    if executed:
        per_div, src = division_valu()
        if per_div is None:
            return None
    tops = (ops_nodiv + div_count * per_div) * n_models / (k_ms / 1e3) / 1e12
    out = {"achieved": tops, "peak": VALU_PEAK_TOPS, "frac": tops / VALU_PEAK_TOPS,
           "unit": "T int32-ops/s"}
    if executed:
        out.update({"valu_per_division": per_div, "source": src})
    return out


if __name__ == "__main__":
    main()
