"""The multi-GPU exchange (mythril_amd/dist.py) with world_size 2 on the gloo
backend (CPU): sharding, coverage OR all-gather, model all-gather with unequal
counts, max/sum timing reduction — the code bench.py runs over RCCL."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mythril_amd import dist as mdist
        res = {}
        res["shard"] = mdist.shard(list(range(10)), rank, world)
        cov = np.zeros(12, dtype=np.uint8)
        cov[rank::3] = 1
        res["cov"] = mdist.allgather_coverage(cov).tolist()
        models = np.full((rank + 1, 2, 8), rank + 7, dtype=np.uint32)
        res["models"] = mdist.allgather_models(models).tolist()
        res["timing"] = mdist.reduce_timing(1.0 + rank, 100.0 * (rank + 1))
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_two_rank_exchange_on_gloo():
    world, port = 2, _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        r0, r1 = out[0], out[1]
    assert r0["shard"] == [0, 2, 4, 6, 8] and r1["shard"] == [1, 3, 5, 7, 9]
    want = [1 if (k % 3) in (0, 1) else 0 for k in range(12)]
    assert r0["cov"] == r1["cov"] == want
    models = np.array(r0["models"])
    assert models.shape == (3, 2, 8) and (models[0] == 7).all() and (models[1:] == 8).all()
    assert r0["models"] == r1["models"]
    assert r0["timing"] == r1["timing"] == (2.0, 300.0)


def _model_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mythril_amd.laser.sharded import exchange_models
        from mythril_amd.smt.program import ArrayInterp, FuncInterp
        from mythril_amd.smt.solver import Model, ModelCache
        mc = ModelCache(device=object())
        own = Model({"x": 5 + rank, "Storage": ArrayInterp(rank, {1: 2}),
                     "keccak256_512": FuncInterp(0, {(7 + rank,): 9})})
        mc.put(own, 1)
        got = exchange_models(mc)
        again = exchange_models(mc)          # nothing new: peers' models are not re-shared
        pool = list(mc.model_cache.lru_cache)
        out[rank] = (got, again, [m.raw[0].assignment["x"] for m in pool],
                     [m.raw[0].assignment["Storage"].default for m in pool],
                     [dict(m.raw[0].assignment["keccak256_512"].entries) for m in pool])
    finally:
        dist.destroy_process_group()


def test_model_allgather_feeds_every_candidate_pool():
    """newly found satisfying models join every rank's ModelCache."""
    world, port = 3, _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_model_worker, args=(world, port, out), nprocs=world, join=True)
        res = [out[r] for r in range(world)]
    for rank, (got, again, xs, defaults, ents) in enumerate(res):
        assert got == world - 1 and again == 0
        assert xs[0] == 5 + rank                           # own model first (put first)
        assert sorted(xs) == [5, 6, 7]
        assert xs[1:] == [5 + r for r in range(world) if r != rank]   # peers in rank order
        assert sorted(defaults) == [0, 1, 2]
        assert all({(7 + r,): 9} in ents for r in range(world))


def _a2a_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mythril_amd import dist as mdist
        # rank r sends q bytes of value 10 r + q to rank q (nothing to itself when q = 0)
        blobs = [bytes([10 * rank + q]) * q for q in range(world)]
        out[rank] = [list(b) for b in mdist.alltoall_bytes(blobs)]
    finally:
        dist.destroy_process_group()


def test_alltoall_bytes_delivers_each_payload_to_its_rank():
    """rebalance's exchange (laser/sharded.py): payload q of rank r arrives at
    rank q as entry r, empty payloads included, at 2 and 3 ranks."""
    for world in (2, 3):
        port = _free_port()
        with mp.Manager() as m:
            out = m.dict()
            mp.spawn(_a2a_worker, args=(world, port, out), nprocs=world)
            got = dict(out)
        for q in range(world):
            assert got[q] == [[10 * r + q] * q for r in range(world)]
