"""Multi-GPU plumbing of the batched core: one process per GPU,
``torch.distributed`` with the nccl (= RCCL over xGMI) backend on the GPU box
and gloo on CPU for the tests.

What crosses ranks is small and latency-bound, so every exchange is one
single-step collective:

* coverage bytes (coverage_plugin.py semantics: a bit is set if any rank
  executed the instruction) — all-gather + OR;
* newly found satisfying models for every rank's candidate pool (kernel 2);
* timing / counters of the benchmark — max of the elapsed times, sum of work.

Work is partitioned without any data-path collective: kernel-1 lanes are
independent paths (each rank runs its own batch / its shard of open states,
split at transaction boundaries, svm.py:239-275); kernel-2 DAG chunks are dealt
round-robin with the model pool replicated.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def rank_world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _device():
    import torch
    import torch.distributed as dist
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" \
        else torch.device("cpu")


def shard(items: Sequence, rank: int, world: int) -> List:
    """Round-robin shard of a work list (open world states at a transaction
    boundary, lane batches, DAG chunks): item k goes to rank k % world."""
    return [x for k, x in enumerate(items) if k % world == rank]


def allgather_coverage(cov: np.ndarray) -> np.ndarray:
    """OR of every rank's coverage bytes for one code (equal lengths)."""
    import torch
    import torch.distributed as dist
    rank, world = rank_world()
    if world == 1:
        return cov.astype(np.uint8)
    t = torch.from_numpy(np.ascontiguousarray(cov, dtype=np.uint8)).to(_device())
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return torch.stack(parts).amax(0).cpu().numpy()


def allgather_models(values: np.ndarray) -> np.ndarray:
    """Concatenate every rank's new candidate models ([k_r, n_vars, 8] u32 limbs,
    k_r may differ per rank) in rank order."""
    import torch
    import torch.distributed as dist
    rank, world = rank_world()
    if world == 1:
        return values
    dev = _device()
    n = torch.tensor([values.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    k_max = max(counts)
    pad = np.zeros((k_max,) + values.shape[1:], dtype=np.uint32)
    pad[: values.shape[0]] = values
    t = torch.from_numpy(pad.view(np.int32)).to(dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    out = [p.cpu().numpy().view(np.uint32)[:c] for p, c in zip(parts, counts)]
    return np.concatenate(out, axis=0)


def alltoall_bytes(blobs: Sequence[bytes]) -> List[bytes]:
    """Point-to-point exchange of byte payloads: ``blobs[q]`` goes to rank q, the
    result's entry r is what rank r sent here.  Two all-to-alls (the sizes, then
    the bytes with per-rank split sizes): every payload crosses the fabric once,
    between the two ranks that need it -- on xGMI a direct link per pair --
    instead of every rank receiving every rank's outgoing states."""
    import torch
    import torch.distributed as dist
    rank, world = rank_world()
    if world == 1:
        return [bytes(blobs[0])] if blobs else [b""]
    dev = _device()
    sizes = torch.tensor([len(b) for b in blobs], dtype=torch.int64, device=dev)
    got = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(got, sizes)
    send_sz, recv_sz = [len(b) for b in blobs], [int(x) for x in got.cpu().tolist()]
    buf = np.frombuffer(b"".join(bytes(b) for b in blobs), dtype=np.uint8) if sum(send_sz) else \
        np.zeros(0, dtype=np.uint8)
    send = torch.from_numpy(buf.copy()).to(dev)
    recv = torch.empty(sum(recv_sz), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=recv_sz, input_split_sizes=send_sz)
    data = recv.cpu().numpy().tobytes()
    out, at = [], 0
    for n in recv_sz:
        out.append(data[at: at + n])
        at += n
    return out


def reduce_timing(elapsed: float, work: float) -> Tuple[float, float]:
    """(max elapsed over ranks, total work over ranks): whole-job throughput =
    total / max (bench.py contract)."""
    import torch
    import torch.distributed as dist
    rank, world = rank_world()
    if world == 1:
        return elapsed, work
    dev = _device()
    mx = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    sm = torch.tensor([work], dtype=torch.float64, device=dev)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return float(mx.item()), float(sm.item())
