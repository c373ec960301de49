"""Multi-process (gloo, world_size 2) rehearsal of bench.py's N>1 structure:
streams sharded by rank, no data-path collective, MAX-over-ranks timing, and
sharded results identical to the single-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard(rank, world, total):
    """Global stream ids of a rank (bench.py: rank * S + i, S = total / world)."""
    per = total // world
    return list(range(rank * per, (rank + 1) * per))


def _worker(rank, world, port, model, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_py
    from conftest import perturbed_stream
    import bench
    base = bench.load_wave()
    m = oracle_py.OracleModel(model)
    res = {}
    dist.barrier()
    import time
    t0 = time.perf_counter()
    for sid in shard(rank, world, 4):
        res[sid] = m.recognize(perturbed_stream(base, sid, seconds=1.5))["path"].tolist()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    gathered = [None] * world
    dist.all_gather_object(gathered, res)
    if rank == 0:
        merged = {}
        for g in gathered:
            merged.update(g)
        out.put((merged, float(el.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_partition():
    for world in (1, 2, 4, 8):
        ids = sum((shard(r, world, 256 * world) for r in range(world)), [])
        assert sorted(ids) == list(range(256 * world))


def test_two_rank_sharding_matches_single_process(synth_model):
    import oracle_py
    from conftest import perturbed_stream
    import bench
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, synth_model, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged, elapsed = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert elapsed > 0
    base = bench.load_wave()
    m = oracle_py.OracleModel(synth_model)
    for sid in range(4):
        ref = m.recognize(perturbed_stream(base, sid, seconds=1.5))["path"].tolist()
        assert merged[sid] == ref
