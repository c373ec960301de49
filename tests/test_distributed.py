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


# ---- admission-time sharding (vosk/shard.py): one int32 all-gather per epoch
def test_plan_admission_prefers_free_capacity():
    from shard import plan_admission
    plan, head = plan_admission([2, 5, 0, 5], 10, 100)
    assert head == 22
    assert [len(p) for p in plan] == [2, 5, 0, 5]
    assert sorted(q for p in plan for q in p) == list(range(10, 22))
    plan, head = plan_admission([3, 3], 0, 4)  # queue shorter than capacity
    assert head == 4 and sorted(plan[0] + plan[1]) == [0, 1, 2, 3]


def _admission_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from shard import AdmissionController
    U, S = 40, 4
    ctl = AdmissionController(dist, U)
    free, active, got = S, {}, []
    step = 0
    while True:
        for u in ctl.admit(free):
            free -= 1
            # rank 0 drains streams 3x faster than rank 1
            active[u] = (1 + u % 3) * (1 if rank == 0 else 3)
            got.append(u)
        done = ctl.gather([len(active), int(ctl.exhausted)])
        if all(a == 0 and x == 1 for a, x in done):
            break
        for u in list(active):
            active[u] -= 1
            if active[u] == 0:
                del active[u]
                free += 1
        step += 1
        assert step < 10000
    out[rank] = got
    dist.destroy_process_group()


def test_admission_controller_gloo_world2():
    """Every utterance is admitted exactly once, both ranks stop together,
    and the faster rank takes more of the queue."""
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_admission_worker, args=(2, port, out), nprocs=2, join=True)
    a, b = out[0], out[1]
    assert sorted(a + b) == list(range(40))
    assert len(a) > len(b)


def test_library_admission_exactly_once_over_two_lanes():
    """The batch path's in-library admission (BatchModel::Admit's PickLane,
    replayed host-only over 2 virtual GPU lanes): every stream is admitted to
    exactly one lane, loads stay balanced, and a lane that drains faster takes
    more streams."""
    from vosk import engine
    rng = np.random.default_rng(5)
    chunks = rng.integers(10, 120, size=400)
    even = engine.admission_replay([40, 40], chunks)
    assert len(even) == len(chunks) and set(even.tolist()) <= {0, 1}
    assert abs(int((even == 0).sum()) - int((even == 1).sum())) <= 20
    fast = engine.admission_replay([60, 20], chunks)
    assert len(fast) == len(chunks)
    assert (fast == 0).sum() > 1.5 * (fast == 1).sum()
    # equal loads: fewest streams, then the lower index
    assert engine.admission_replay([0, 0], [5, 5, 5, 5]).tolist() == [0, 1, 0, 1]


# ---- the product path over two processes (one BatchModel lane each)
def _lane_worker(rank, world, port, model, nstreams, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VOSK_AMD_DEVICE="0",
                      VOSK_BATCH_MODEL_DIR=model)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = _batch_texts(shard(rank, world, nstreams))
    gathered = [None] * world
    dist.all_gather_object(gathered, res)
    if rank == 0:
        merged = {}
        for g in gathered:
            merged.update(g)
        out.put(merged)
    dist.barrier()
    dist.destroy_process_group()


def _batch_texts(ids):
    """Every result message of each stream, through libvosk.so's batch API
    (the test_gpu_batch.py loop), for the global stream ids `ids`."""
    import json
    import vosk
    import bench
    from conftest import perturbed_stream
    vosk.SetLogLevel(-1)
    base = bench.load_wave()
    datas = {i: bench.pcm(perturbed_stream(base, 4000 + i, seconds=4.0 + 0.5 * i)) for i in ids}
    vosk.GpuInit()
    bm = vosk.BatchModel()
    recs = {i: vosk.BatchRecognizer(bm, 16000) for i in ids}
    got = {i: [] for i in ids}

    def collect():
        for i in ids:
            while True:
                r = recs[i].Result()
                if not r:
                    break
                got[i].append(json.loads(r))
    n = max(len(d) for d in datas.values())
    for pos in range(0, n, 8000):
        for i in ids:
            if pos < len(datas[i]):
                recs[i].AcceptWaveform(datas[i][pos:pos + 8000])
        bm.Wait()
        collect()
    for i in ids:
        recs[i].FinishStream()
    bm.Wait()
    collect()
    del recs
    del bm
    return got


@pytest.mark.gpu
def test_two_processes_of_batch_lanes_match_oracle(synth_model, test_wave):
    """bench.py's N > 1 structure on the product path: two processes (gloo
    world 2), each with its own libvosk.so BatchModel lane (both on device 0
    here, one GPU per rank on a node) decoding its shard of the streams; the
    gathered results equal the oracle's for every stream
    (tests/batch_expect.py: segments, words and times)."""
    import batch_expect
    from conftest import perturbed_stream
    n = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lane_worker, args=(r, 2, port, synth_model, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(merged) == list(range(n))
    waves = [perturbed_stream(test_wave, 4000 + i, seconds=4.0 + 0.5 * i) for i in range(n)]
    exp = batch_expect.expected(synth_model, waves)
    for i in range(n):
        batch_expect.check(merged[i], exp[i], f"stream {i}")
