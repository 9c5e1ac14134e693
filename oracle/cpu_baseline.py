"""CPU baseline of bench.py (TEST INFRASTRUCTURE ONLY): the C oracle, timed on host cores.

The reference (Python LASER + z3) cannot run on the GPU box (not importable, and
the reference never travels there), so the comparator is the oracle's C port of
the same semantics (``kind: "port"``), -O3, one pthread per core over disjoint
lanes.  Bounded sample: the C2 lane batch is re-run from its initial image until
about `seconds` of CPU time has elapsed.
"""
import ctypes
import os
import time

from . import lib
from .evm_ref import OracleEVM


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _usable_cores():
    """CPUs this process may run on (its affinity mask)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cpu_share():
    """The threads the comparator uses: every usable core, unless the host
    states this job's CPU share (OMP_NUM_THREADS -- the GPU box sets it to the
    share of one GPU, 16, and asks worker pools to stay within it)."""
    n = _usable_cores()
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        share = 0
    return min(n, share) if share > 0 else n


def _cores_info(threads: int) -> dict:
    return {"cores": threads, "usable_cores": _usable_cores(), "host_cpus": os.cpu_count(),
            "cpu_share_env": os.environ.get("OMP_NUM_THREADS"), "cpu_model": _cpu_model()}


def c2_lane_steps(code: bytes, seconds: float = 10.0, lanes: int = 65536, threads: int = 0) -> dict:
    from mythril_amd import workloads
    o = OracleEVM()
    cid = o.load_code(code)
    base = workloads.c2_batch(lanes, code_id=cid, stack_cap=64, mem_cap=1024, rec_cap=128)
    threads = threads or _cpu_share()
    mask = (ctypes.c_uint64 * 4)(0, 0, 0, 0)
    lib().orc_run_mt.restype = ctypes.c_uint64
    lib().orc_run_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]

    def timed(nthreads, budget):
        steps, el, reps = 0, 0.0, 0
        while el < budget or reps == 0:
            b = base.copy()
            soa = b.soa()
            t0 = time.perf_counter()
            steps += int(lib().orc_run_mt(ctypes.addressof(soa), 0, b.n, mask, 1 << 30, 0, nthreads))
            el += time.perf_counter() - t0
            reps += 1
        return steps / el, reps

    single, reps1 = timed(1, min(seconds / 3, 5.0))
    multi, repsn = timed(threads, seconds)
    return {"value": multi, "unit": "lane-steps/s", **_cores_info(threads), "kind": "port",
            "sample": f"C2 batch ({lanes} lanes, overflow.sol.o) x {repsn} runs on {threads} threads; "
                      f"C oracle oracle/evm_ref.c -O3 ({_cpu_model()})",
            "single_core_value": single}


def c4_evals(n_models: int = 4096, seconds: float = 10.0, threads: int = 0) -> dict:
    """C4 constraint-evals/s of oracle/bv_ref.c on a bounded sample of DAGs (all
    models), one pthread per core."""
    from mythril_amd.smt import synth
    from .bv_ref import eval_batch
    threads = threads or _cpu_share()
    models = synth.c4_models(n_models, synth.C4_SEED + 0x1000)
    prog = synth.c4_programs(synth.Draws(4096, synth.C4_SEED))
    done, el, d = 0, 0.0, 0
    while el < seconds and d < prog.n_dags:
        cnt = min(threads * 8, prog.n_dags - d)
        t0 = time.perf_counter()
        eval_batch(prog, models, first=d, count=cnt, threads=threads)
        el += time.perf_counter() - t0
        done += cnt * n_models
        d += cnt
    return {"value": done / el, "unit": "constraint-evals/s", **_cores_info(threads), "kind": "port",
            "sample": f"{d} C4 DAGs x {n_models} models on {threads} threads; oracle/bv_ref.c -O3 "
                      f"({_cpu_model()})"}
