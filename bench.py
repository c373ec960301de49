#!/usr/bin/env python3
"""Aggregate real-time factor of the Vosk batch path on MI355X.

Headline workload (BASELINE.json configs[2], the largest single-GPU
configuration): the reference's own GPU batch harness,
python/example/test_gpu_batch.py:25-59, through the public API -- 256
BatchRecognizers per GPU fed 8000-byte s16le chunks from host memory, one
feeding round over every stream, BatchModel.Wait(), Result() of every stream
-- on 60 s streams.  libvosk.so's BatchModel runs one GPU lane per process
here (VOSK_AMD_DEVICE = LOCAL_RANK): MFCC + online i-vectors -> looped TDNN-F
nnet3 (fp32 MFMA) -> token passing (beam 13, max-active 7000) with lattices
-> endpointing -> lattice MBR results on host worker threads.  A "step" is
one feeding round (0.25 s of audio per stream); the timed region also covers
FinishStream, the last Wait and the final results.

Model: no Vosk model is available offline, so a seeded synthetic model in
the real Kaldi/OpenFST formats stands in for vosk-model-small-en-us: the
recipe's TDNN-F topology (training/local/chain/run_tdnn.sh:98-129, random-init
weights, BatchNorm calibrated on test.wav) with a 20 k-word lookahead graph
(HCLr + a ~29 k-history trigram Gr, expanded at load to ~275 k states).
Streams are test.wav tiled, shifted, gained and noised per BASELINE.md.

Secondary keys: "engine_only" (the GPU engine stepped directly on
HBM-resident audio, no host feeding or result production), the single-stream
KaldiRecognizer latency (config 2), 32 KaldiRecognizers on 32 threads
("concurrent_recognizers": their calls share batched engine passes),
"round_parts_ms" (feed / Wait / collect per round), "result_production"
(lattice copy / build / determinize / MBR totals and the lane's host time)
and the CPU baseline.

Multi-GPU: one process per GPU (torchrun); streams are sharded by rank with
no data-path collective ("scaling": "weak"); a barrier brackets the timed
region and the MAX elapsed time over ranks is used.
"""
import argparse
import json
import os
import sys
import time
import wave

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "vosk-api_amd")
for _p in (PKG, os.path.join(PKG, "tools"), os.path.join(REPO, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3   # dense fp32 MFMA peak (MI355X_MICROARCH.md)
SR = 16000
FEED_BYTES = 8000          # test_gpu_batch.py:33 reads 8000 bytes per stream per round
METRIC = "aggregate real-time factor (xRT) + p50 per-chunk latency, vosk-model-small-en-us"
PMC_PROFILE = os.path.join(REPO, "profiles", "r06_final_decode_pmc.json")


def load_wave():
    w = wave.open(os.path.join(REPO, "tests", "golden", "test.wav"), "rb")
    return np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)


def stream_audio(base, i, n):
    from conftest import perturbed_stream
    return perturbed_stream(base, i, seconds=n / SR)


def pcm(x):
    return np.clip(np.asarray(x, np.float32), -32768, 32767).astype("<i2").tobytes()


def bench_model(rank, dist, preset):
    import make_synth_model
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), "vamd_models", f"bench_{preset}_v4")
    if rank == 0 and not os.path.exists(os.path.join(cache, "README")):
        tmp = cache + f".tmp{os.getpid()}"
        make_synth_model.make_preset(preset, tmp)
        os.rename(tmp, cache)
    if dist is not None:
        dist.barrier()
    return cache


def cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return os.cpu_count() or 1, model


def cpu_workers():
    """Host cores this process may use: its affinity set, capped by the
    box's CPU share when the environment states one (OMP_NUM_THREADS)."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_baseline(model, base, streams, seconds, workers):
    """Oracle (single-threaded C restatement: MFCC, i-vectors, nnet3, token
    passing) timed on host cores: one stream per worker process at a time
    (the transcribe_scp.py Pool pattern)."""
    import multiprocessing as mp
    jobs = [(i, seconds) for i in range(streams)]
    ctx = mp.get_context("fork")
    with ctx.Pool(workers, initializer=_cpu_init, initargs=(model,)) as pool:
        t0 = time.time()
        res = pool.map(_cpu_job, jobs, chunksize=1)
        wall = time.time() - t0
    audio = sum(r[0] for r in res)
    return audio / wall, audio, wall


_ORC = {}


def _cpu_init(model):
    import oracle_py
    _ORC["m"] = oracle_py.OracleModel(model, fpc=51)  # the batch chunking (i-vector per chunk)
    _ORC["base"] = load_wave()


def _cpu_job(args):
    i, seconds = args
    x = stream_audio(_ORC["base"], 10_000 + i, int(seconds * SR))
    t = time.time()
    _ORC["m"].recognize(x)
    return len(x) / SR, time.time() - t


def oracle_model_dir(model):
    """The oracle reads graph/HCLG.fst: for a lookahead model, a copy with
    libvosk's static expansion of HCLr o Gr (the graph the GPU decodes)."""
    if os.path.exists(os.path.join(model, "graph", "HCLG.fst")):
        return model
    import oracle_graph as OG
    out = model.rstrip("/") + "_oracle_hclg"
    if not os.path.exists(os.path.join(out, "graph", "lazy_ids.npz")):
        OG.expanded_hclg_model(model, out + ".tmp")
        __import__("shutil").rmtree(out, ignore_errors=True)
        os.rename(out + ".tmp", out)
    return out


def decoder_roofline(dec_ms, dec_launches, tot, kernel):
    """HBM roofline of the decoder launches: algorithmic bytes (SURVEY.md 8d,
    16*T_in + 24*E + 16*T_new + 20*L_bp + 16 per lattice link) per launch over
    the HIP-event launch time on the decoder's stream."""
    E = tot["arcs_emit"] + tot["arcs_eps"]
    alg = 16 * tot["tok_in"] + 24 * E + 16 * tot["tok_out"] + 20 * tot["tok_out"] + 16 * tot.get("links", 0)
    n = max(dec_launches, 1)
    launch_ms = dec_ms / n
    gbs = (alg / n) / (launch_ms * 1e-3) / 1e9 if dec_ms > 0 else 0.0
    traffic, source = None, None
    if os.path.exists(PMC_PROFILE):
        try:
            traffic = json.load(open(PMC_PROFILE)).get("hbm_bytes_per_launch")
            source = os.path.relpath(PMC_PROFILE, REPO) + " (rocprofv3 FETCH_SIZE+WRITE_SIZE passes)"
        except Exception:
            traffic = None
    return {"bound": "hbm", "kernel": kernel, "achieved": round(gbs, 3), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": source,
            "avg_launch_ms": round(launch_ms, 4), "launches": dec_launches,
            "alg_bytes_per_launch": alg / n}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed feeding rounds (0.25 s per stream each); default: the rest of "
                         "--stream-seconds after the warmup")
    ap.add_argument("--warmup", type=int, default=8, help="untimed feeding rounds")
    ap.add_argument("--stream-seconds", type=float, default=60.0)
    ap.add_argument("--streams", type=int, default=256, help="streams per GPU")
    ap.add_argument("--preset", default="la_small_en_us", help="synthetic model preset")
    ap.add_argument("--model", default=None, help="model directory (overrides --preset)")
    ap.add_argument("--workload", choices=("api", "engine", "dynamic", "spk"), default="api",
                    help="api (default, the headline): test_gpu_batch.py through vosk_batch_*; "
                         "engine: the GPU engine stepped on HBM-resident audio; dynamic: "
                         "variable-length utterances admitted per epoch across ranks; spk: "
                         "config 5's speaker path, batched x-vector extraction")
    ap.add_argument("--engine-steps", type=int, default=20)
    ap.add_argument("--no-engine-line", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single-stream", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true")
    ap.add_argument("--no-lattice", action="store_true")
    ap.add_argument("--order", choices=("parallel", "kaldi"), default="kaldi",
                    help="engine workloads: token-passing order (kaldi = the CPU reference's "
                         "LatticeFasterDecoder order, the BatchModel lanes' default)")
    ap.add_argument("--no-order-line", action="store_true",
                    help="skip the secondary API line in the other token-passing order")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU baseline: seconds per stream")
    ap.add_argument("--lanes", default=None,
                    help="in-library lanes mode (one process, no torchrun): the BatchModel runs one lane "
                         "per listed device (VOSK_AMD_BATCH_DEVICES, e.g. 0,1,2,3,4,5,6,7 or 0,0), "
                         "--streams per lane, admission by the library's PickLane")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if args.lanes:
        if world > 1:
            raise SystemExit("bench.py --lanes runs as one process (the library drives every lane)")
        os.environ["VOSK_AMD_BATCH_DEVICES"] = args.lanes
        os.environ.pop("VOSK_AMD_DEVICE", None)
    else:
        os.environ["VOSK_AMD_DEVICE"] = str(local_rank)  # one BatchModel lane (GPU) per rank
    # torchrun exports OMP_NUM_THREADS=1 to every rank when the environment
    # sets none; the library caps its result workers by it (it reads it as the
    # process's CPU share), which would leave each rank two workers for the
    # final segments' lattices.  Give each rank its share of this node's cores
    # instead (at most the 16 of a one-GPU box).
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    if world > 1 and os.environ.get("OMP_NUM_THREADS") == "1" and "VOSK_AMD_RESULT_THREADS" not in os.environ:
        share = max(2, min(16, len(os.sched_getaffinity(0)) // max(local_world, 1)))
        os.environ["VOSK_AMD_RESULT_THREADS"] = str(max(2, share - 1))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend=backend)
        dist = tdist

    if args.workload == "spk":
        return run_spk(args, dist, rank, world)
    model = args.model or bench_model(rank, dist, args.preset)
    import vosk
    from vosk import engine as ve
    vosk.SetLogLevel(-1)
    if ve.device_count() == 0:
        raise SystemExit("bench.py: no HIP device visible")
    if args.workload == "dynamic":
        return run_dynamic(args, model, dist, rank, world)
    base = load_wave()
    if args.workload == "engine":
        out = run_engine(args, model, dist, rank, world, base, args.steps or 40)
    else:
        out = run_api(args, model, dist, rank, world, base)
        if not args.no_order_line:
            # the same workload with the lanes in the other token-passing order
            # (VOSK_AMD_DEC_ORDER is read when the BatchModel's engines are built)
            other = "parallel" if (out or {}).get("decoder_order", "kaldi") == "kaldi" else "kaldi"
            os.environ["VOSK_AMD_DEC_ORDER"] = other
            try:
                alt = run_api(args, model, dist, rank, world, base)
            finally:
                os.environ.pop("VOSK_AMD_DEC_ORDER", None)
            if alt is not None:
                key = "kaldi_order" if other == "kaldi" else "order_independent"
                out[key] = {k: alt[k] for k in ("value", "unit", "ms_per_step", "finish_ms", "decoder_order",
                                                "p50_chunk_latency_ms", "p99_chunk_latency_ms", "roofline",
                                                "gpu_ms_per_step", "decoder", "results")}
        if not args.no_engine_line:
            eng = run_engine(args, model, dist, rank, world, base, args.engine_steps)
            if eng is not None:
                out["engine_only"] = {k: eng[k] for k in ("value", "unit", "ms_per_step", "steps",
                                                          "stages_ms_per_step", "roofline",
                                                          "roofline_nnet", "decoder", "config")}
    if rank == 0 and world == 1:
        if not args.no_single_stream:
            out["single_stream"] = single_stream_latency(model, base)
            out["concurrent_recognizers"] = concurrent_recognizers_child(model)
        if not args.no_cpu_baseline:
            nproc, cpu_model = cpu_info()
            workers = cpu_workers()
            odir = oracle_model_dir(model)
            v, a, w = cpu_baseline(odir, base, workers, args.cpu_seconds, workers)
            out["cpu_baseline"] = {
                "value": round(v, 3), "unit": "xRT", "cores": workers, "kind": "port",
                "nproc": nproc, "cpu_model": cpu_model,
                "sample": f"{workers} synthetic streams x {args.cpu_seconds:.0f} s through the C oracle "
                          f"(MFCC + i-vectors + nnet3 + token passing on the same graph), one stream per "
                          f"worker process, {workers} processes (affinity/OMP share of {nproc} CPUs), "
                          f"{a:.0f} s audio in {w:.1f} s wall.  Not the same work as the GPU line: no "
                          f"lattices, endpointing, determinization or MBR results on this leg"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _max_over_ranks(dist, elapsed):
    if dist is None:
        return elapsed
    import torch
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run_api(args, model, dist, rank, world, base):
    """test_gpu_batch.py:25-59 on S streams per GPU: feed 8000 bytes to every
    stream, Wait(), Result() of every stream; FinishStream at the end."""
    import vosk
    from vosk import engine as ve
    lanes = [int(x) for x in args.lanes.split(",") if x] if args.lanes else [0]
    S = args.streams * len(lanes)
    W = args.warmup
    K = args.steps if args.steps is not None else max(1, int(round(args.stream_seconds * SR * 2 / FEED_BYTES)) - W)
    rounds = W + K
    os.environ["VOSK_BATCH_MODEL_DIR"] = model
    os.environ["VOSK_AMD_BATCH_TIMING"] = "1"   # HIP-event stage times on the lane's streams
    os.environ["VOSK_AMD_BATCH_STATS"] = "1"    # decoder work counters (roofline bytes)
    if args.no_pipeline:
        os.environ["VOSK_AMD_BATCH_PIPELINE"] = "0"
    datas = [pcm(stream_audio(base, rank * S + i, rounds * FEED_BYTES // 2)) for i in range(S)]
    vosk.GpuInit()
    bm = vosk.BatchModel()
    recs = [vosk.BatchRecognizer(bm, SR) for _ in range(S)]
    texts = [""] * S
    nres = [0]

    def collect():
        for i in range(S):
            res = recs[i].Result()
            if res:
                texts[i] = texts[i] + " " + json.loads(res)["text"]
                nres[0] += 1

    parts = {True: np.zeros(3), False: np.zeros(3)}  # chunk round? -> feed, wait, collect seconds
    nparts = {True: 0, False: 0}
    spc = 8160 * 2  # bytes per 51-frame chunk (samples_per_chunk, batch_model.cc:84-88)

    def feed_round(k):
        o = k * FEED_BYTES
        t0 = time.perf_counter()
        for i in range(S):
            recs[i].AcceptWaveform(datas[i][o:o + FEED_BYTES])
        t1 = time.perf_counter()
        bm.Wait()
        t2 = time.perf_counter()
        collect()
        t3 = time.perf_counter()
        kind = ((k + 1) * FEED_BYTES) // spc > (k * FEED_BYTES) // spc
        parts[kind] += (t1 - t0, t2 - t1, t3 - t2)
        nparts[kind] += 1

    for k in range(W):
        feed_round(k)
    for kind in parts:
        parts[kind][:] = 0
        nparts[kind] = 0
    for lane in range(ve.batch_lanes(bm)):
        ve.batch_lane_stats(bm, lane, reset=True)
    if dist is not None:
        dist.barrier()
    lat = []
    t0 = time.perf_counter()
    for k in range(W, rounds):
        ts = time.perf_counter()
        feed_round(k)
        # rounds that complete a chunk: Push -> results of the round available
        if ((k + 1) * FEED_BYTES) // spc > (k * FEED_BYTES) // spc:
            lat.append(time.perf_counter() - ts)
    tf = time.perf_counter()
    for r in recs:
        r.FinishStream()
    bm.Wait()
    collect()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    elapsed = _max_over_ranks(dist, t1 - t0)
    audio_s = K * FEED_BYTES / 2 / SR * S * world
    nl = ve.batch_lanes(bm)
    order = ve.batch_lane_order(bm, 0)
    lane_streams = [sum(1 for r in recs if ve.batch_recognizer_lane(r) == li) for li in range(nl)]
    st = ve.batch_lane_stats(bm, 0)
    mem = ve.batch_lane_memory(bm, 0)
    rprof = ve.batch_result_profile(bm)
    nonempty = sum(1 for t in texts if t.strip())
    words = sum(len(t.split()) for t in texts)
    del recs
    del bm
    if rank != 0:
        return None
    dec_ms, dec_n = st["stages"]["decode"]
    nnet_ms, nnet_n = st["stages"]["nnet"]
    front_ms, _ = st["stages"]["front"]
    step_ms, steps = st["stages"]["step"]
    tot = st["decoder"]
    info = ve.plan_info(model, 51)
    opc = 51 // 3
    nnet_flops = tot["frames"] / opc * info["flops_per_chunk"]
    nnet_tflops = nnet_flops / (nnet_ms * 1e-3) / 1e12 if nnet_ms else 0.0
    lat_ms = np.array(lat) * 1e3 if lat else np.zeros(1)
    return {
        "metric": METRIC, "value": round(audio_s / elapsed, 2), "unit": "xRT",
        "n_gpus": len(set(lanes)) if args.lanes else world,
        "steps": K, "warmup": W, "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic: test.wav tiled/shifted/gain/noise per BASELINE.md, s16le host buffers; "
                "seeded random-init synthetic model (recipe TDNN-F topology, 20k-word lookahead "
                "HCLr + trigram Gr expanded to a static graph)",
        "config": {"workload": "config3: test_gpu_batch.py loop through vosk_batch_* (BatchModel + "
                               "BatchRecognizer, 8000-byte feeds, Wait, Result per round), "
                               f"{args.streams} streams/lane x {rounds * FEED_BYTES / 2 / SR:.0f} s, "
                               + (f"one process, in-library lanes on devices {args.lanes}" if args.lanes
                                  else "1xMI355X per rank"),
                   "model": os.path.basename(model.rstrip("/")), "streams_per_gpu": args.streams,
                   "global_streams": S * world, "feed_bytes": FEED_BYTES, "chunk_samples": 8160,
                   "frames_per_chunk": 51, "beam": 13.0, "max_active": 7000, "lattice_beam": 6.0,
                   "parallelism": f"lanes{len(lanes)}" if args.lanes else f"dp{world}",
                   "lane_streams": lane_streams,
                   "pipeline": "lane thread: front(s) || nnet(s-1) || decoder(s-2) on 3 HIP streams "
                               "while chunks are queued; a round with nothing behind it runs its "
                               "stages in order; MBR results on host worker threads"},
        "decoder_order": order,
        "decoder_order_note": ("kaldi: LatticeFasterDecoder's sequential token passing, the CPU reference's "
                               "1-best (DESIGN.md §4); parallel: the order-independent form"),
        "step": "one feeding round: 8000 bytes to every stream, Wait(), Result() of every stream",
        "timed_region": "rounds W..W+K, then FinishStream + Wait + final results",
        "p50_chunk_latency_ms": round(float(np.percentile(lat_ms, 50)), 3),
        "p90_chunk_latency_ms": round(float(np.percentile(lat_ms, 90)), 3),
        "p99_chunk_latency_ms": round(float(np.percentile(lat_ms, 99)), 3),
        "latency_definition": "wall time of a feeding round that completes a chunk: AcceptWaveform "
                              "(Push) of every stream -> Wait() -> results collected",
        "finish_ms": round((t1 - tf) * 1e3, 3),
        "round_parts_ms": {("chunk_rounds" if kind else "other_rounds"): {
            "rounds": nparts[kind], **{n: round(float(v) / max(nparts[kind], 1) * 1e3, 3)
                                       for n, v in zip(("feed", "wait", "collect"), parts[kind])}}
            for kind in (True, False)},
        "roofline": decoder_roofline(dec_ms, dec_n, tot, "decode_kernel"),
        "roofline_nnet": {"bound": "mfma", "kernel": "nnet GEMM launches", "achieved": round(nnet_tflops, 4),
                          "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": nnet_tflops / FP32_PEAK_TFLOPS},
        "gpu_ms_per_step": {"front": round(front_ms / K, 4), "nnet": round(nnet_ms / K, 4),
                            "decode": round(dec_ms / K, 4), "engine_steps": steps},
        "decoder": {"frames": tot["frames"],
                    "tokens_per_frame": round(tot["tok_out"] / max(tot["frames"], 1), 1),
                    "arcs_per_frame": round((tot["arcs_emit"] + tot["arcs_eps"]) / max(tot["frames"], 1), 1),
                    "lattice_links_per_frame": round(tot["links"] / max(tot["frames"], 1), 1)},
        "lane_memory": mem,
        "results": {"streams_with_text": nonempty, "words": words, "result_messages": nres[0]},
        "result_production": {k: round(v, 2) for k, v in rprof.items()},
    }


def run_engine(args, model, dist, rank, world, base, steps):
    """The GPU engine stepped directly: every step advances all S streams by
    one 8160-sample chunk of HBM-resident audio (no host feeding, no result
    production)."""
    from vosk import engine as ve
    S = args.streams
    pipe = not args.no_pipeline
    warm = 5
    e = ve.Engine(model, frames_per_chunk=51, max_streams=S, stats=True, time_kernels=True,
                  pipeline=pipe, lattice=not args.no_lattice, order=args.order)
    chunk = e.fpc * 160
    e.set_step_samples(chunk)
    total_steps = warm + steps + 2
    streams = []
    for i in range(S):
        s = e.new_stream()
        e.preload(s, stream_audio(base, rank * S + i, total_steps * chunk), finished=False)
        streams.append(s)
    for _ in range(warm):
        e.step(streams)
    e.stage_times(reset=True)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        e.step(streams)
    elapsed = _max_over_ranks(dist, time.perf_counter() - t0)
    st = e.stage_times()
    tot = e.decoder_totals()
    errs = sum(1 for s in streams if e.error(s))
    flops = e.flops_per_chunk
    phases = None
    if os.environ.get("VOSK_AMD_DEC_PROFILE"):
        ph = e.decoder_phases()
        phases = {k: round(v / max(ph["frames"], 1), 4) for k, v in ph.items() if k != "frames"}
        per = e.decoder_phases_per_stream()[:S]
        clk = per[:, e.PHASE_CLOCK_IDX].sum(1).astype(np.float64)
        phases["stream_clock_max_over_mean"] = round(float(clk.max() / max(clk.mean(), 1.0)), 3)
    e.close()
    if rank != 0:
        return None
    dec_ms, dec_n = st["decode"]
    nnet_ms, _ = st["nnet"]
    front_ms, _ = st["front"]
    nnet_tflops = flops * S * steps / (nnet_ms * 1e-3) / 1e12 if nnet_ms else 0.0
    out = {
        "metric": METRIC, "value": round(steps * S * chunk / SR * world / elapsed, 2), "unit": "xRT",
        "n_gpus": world, "steps": steps, "warmup": warm, "ms_per_step": round(elapsed / steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (HBM-resident audio), seeded random-init synthetic model",
        "config": {"workload": "engine: GPU engine steps over HBM-resident audio (no host feeding, "
                               "no result production)", "streams_per_gpu": S, "chunk_samples": chunk,
                   "pipeline": "front(s) || nnet(s-1) || decoder(s-2), 3 HIP streams" if pipe else "in-order"},
        "roofline": decoder_roofline(dec_ms, dec_n, tot, "decode_kernel"),
        "roofline_nnet": {"bound": "mfma", "kernel": "nnet GEMM launches", "achieved": round(nnet_tflops, 4),
                          "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": nnet_tflops / FP32_PEAK_TFLOPS},
        "stages_ms_per_step": {"front": round(front_ms / steps, 4), "nnet": round(nnet_ms / steps, 4),
                               "decode": round(dec_ms / steps, 4),
                               "gpu_step": round(st["step"][0] / steps, 4)},
        "decoder": {"frames": tot["frames"],
                    "tokens_per_frame": round(tot["tok_out"] / max(tot["frames"], 1), 1),
                    "arcs_per_frame": round((tot["arcs_emit"] + tot["arcs_eps"]) / max(tot["frames"], 1), 1),
                    "lattice_links_per_frame": round(tot.get("links", 0) / max(tot["frames"], 1), 1),
                    "stream_errors": errs},
    }
    if phases is not None:
        out["decoder_phase_clocks_per_frame"] = phases
    return out


def single_stream_latency(model, base, seconds=30.0, chunk_bytes=8000):
    """One KaldiRecognizer (silence-weighted i-vectors, lattice results)
    fed 8000-byte chunks; p50/p90/p99 of the accept_waveform wall time, the
    stream's real-time factor, and a final result call's time."""
    import vosk
    data = pcm(stream_audio(base, 777, int(seconds * SR)))
    m = vosk.Model(model)
    rec = vosk.KaldiRecognizer(m, SR)
    rec.SetWords(True)
    for i in range(0, 16000 * 2, chunk_bytes):  # warm up (first kernels, allocations)
        rec.AcceptWaveform(data[i:i + chunk_bytes])
    rec.FinalResult()
    lat = []
    t0 = time.perf_counter()
    for i in range(0, len(data), chunk_bytes):
        ts = time.perf_counter()
        if rec.AcceptWaveform(data[i:i + chunk_bytes]):
            rec.Result()
        lat.append(time.perf_counter() - ts)
    tf = time.perf_counter()
    rec.FinalResult()
    t1 = time.perf_counter()
    lat = np.array(lat) * 1e3
    return {"p50_accept_ms": round(float(np.percentile(lat, 50)), 3),
            "p90_accept_ms": round(float(np.percentile(lat, 90)), 3),
            "p99_accept_ms": round(float(np.percentile(lat, 99)), 3),
            "final_result_ms": round((t1 - tf) * 1e3, 3),
            "xrt": round(seconds / (t1 - t0), 2),
            "chunk": "8000 B (0.25 s) per accept_waveform, test_simple.py pattern, 30 s stream; "
                     "results (MBR over the GPU lattice) included when an endpoint fires"}


def concurrent_recognizers_child(model, threads=32, seconds=20.0, queues=8):
    """concurrent_recognizers in a process of its own, started with
    GPU_MAX_HW_QUEUES=`queues`: its recognizers are spread over queues / 2
    engines (csrc/vosk_impl.cc StreamEngineSpread), the configuration the
    Python package asks for when the environment sets no number; this
    process's HIP runtime already runs with the environment's count."""
    import subprocess
    env = dict(os.environ)
    env["GPU_MAX_HW_QUEUES"] = str(queues)
    here = os.path.dirname(os.path.abspath(__file__))
    # two runs, the second reported (the first is the process's warm-up, as
    # the headline legs before this one are for the in-process legs)
    cmd = [sys.executable, "-u", os.path.join(here, "tools", "conc_bench.py"), f"{threads},{threads}", str(seconds),
           model]
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        res = json.loads(p.stdout.strip().splitlines()[-1])
    except Exception as e:  # reported, not hidden: the leg's value is missing
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    res["hw_queues"] = queues
    res["process"] = "child process (own HIP runtime), second of two runs"
    return res


def concurrent_recognizers(model, base, threads=32, seconds=20.0, chunk_bytes=8000):
    """`threads` KaldiRecognizers, one per Python thread (vosk-server's
    shape), each fed 8000-byte chunks of its own stream; their engine calls
    are coalesced into shared GPU steps (Engine::AdvanceCoalesced).  Reports
    the aggregate xRT and the per-call latency percentiles."""
    import threading
    import vosk
    datas = [pcm(stream_audio(base, 900 + i, int(seconds * SR))) for i in range(threads)]
    m = vosk.Model(model)
    recs = [vosk.KaldiRecognizer(m, SR) for _ in range(threads)]
    for r in recs:  # warm up every slot
        r.AcceptWaveform(datas[0][:chunk_bytes])
        r.FinalResult()
    lats = [[] for _ in range(threads)]
    go = threading.Barrier(threads + 1)

    def work(i):
        rec, d, lat = recs[i], datas[i], lats[i]
        go.wait()
        for o in range(0, len(d), chunk_bytes):
            ts = time.perf_counter()
            if rec.AcceptWaveform(d[o:o + chunk_bytes]):
                rec.Result()
            lat.append(time.perf_counter() - ts)
        rec.FinalResult()

    th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in th:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    lat = np.concatenate([np.array(x) for x in lats]) * 1e3
    del recs
    return {"threads": threads, "xrt": round(threads * seconds / el, 2),
            "p50_accept_ms": round(float(np.percentile(lat, 50)), 3),
            "p99_accept_ms": round(float(np.percentile(lat, 99)), 3),
            "workload": f"{threads} KaldiRecognizers on {threads} threads, {seconds:.0f} s streams, "
                        "8000-byte accept_waveform calls, Result on endpoints, FinalResult"}


def run_dynamic(args, model, dist, rank, world):
    """Variable-length utterances (5-60 s, seeded) from one node-wide queue
    (3 x streams x GPUs of them), admitted every 4 steps to the ranks with the
    most free slots; a finished stream frees its slot.  Samples are uploaded
    when a stream is admitted (inside the timed region: this mode measures
    the admission path, not the headline)."""
    from vosk import engine as ve
    from shard import AdmissionController
    S = args.streams
    e = ve.Engine(model, frames_per_chunk=51, max_streams=S, stats=True, lattice=not args.no_lattice,
                  order=args.order)
    chunk = e.fpc * 160
    e.set_step_samples(chunk)
    base = load_wave()
    U = 3 * S * world
    rng = np.random.default_rng(99)
    lens = (rng.uniform(5.0, 60.0, size=U) * SR).astype(np.int64)
    dev = "cpu"
    if dist is not None:
        import torch
        dev = "cuda" if torch.cuda.is_available() else "cpu"
    ctl = AdmissionController(dist, U, device=dev)
    wav = {u: stream_audio(base, 50_000 + u, int(lens[u])) for u in range(U)}
    free = [e.new_stream() for _ in range(S)]
    active = {}  # slot -> (utterance, expected decoder frames)
    audio = 0.0
    steps = 0
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    while True:
        if steps % 4 == 0:
            for u in ctl.admit(len(free)):
                s = free.pop()
                e.reset(s)
                x = wav[u]
                e.preload(s, x, finished=True)
                frames = 1 + (len(x) - 400) // 160 if len(x) >= 400 else 0
                active[s] = (u, (frames + 2) // 3)
                audio += len(x) / SR
            done_all = ctl.gather([len(active), int(ctl.exhausted)])
            if all(a == 0 for a, _ in done_all) and all(x == 1 for _, x in done_all):
                break
        if active:
            e.step(list(active))
        steps += 1
        if steps > 1_000_000:
            raise SystemExit("bench.py dynamic: streams did not finish")
        for s in list(active):
            if e.frames_decoded(s) >= active[s][1]:
                del active[s]
                free.append(s)
    elapsed = time.perf_counter() - t0
    tot_audio = audio
    if dist is not None:
        import torch
        elapsed = _max_over_ranks(dist, elapsed)
        a = torch.tensor([audio], dtype=torch.float64, device=dev)
        dist.all_reduce(a, op=dist.ReduceOp.SUM)
        tot_audio = float(a.item())
    if rank == 0:
        print(json.dumps({
            "metric": "aggregate real-time factor (xRT), dynamic admission",
            "value": round(tot_audio / elapsed, 2), "unit": "xRT", "n_gpus": world,
            "steps": steps, "warmup": 0, "ms_per_step": round(1000 * elapsed / max(steps, 1), 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic variable-length utterances (5-60 s) from test.wav",
            "config": {"workload": "dynamic: node-wide queue, admission every 4 steps by int32 "
                                   "all-gather of free slots", "utterances": U,
                       "streams_per_gpu": S, "admission_epochs": ctl.epochs}}), flush=True)
    e.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()



# ---------------------------------------------------------------- config 5
SPK_DIMS = dict(hidden=512, stats_dim=1500, embed=512, out=128)  # the sre16 x-vector recipe's sizes


def spk_bench_model(rank, dist):
    import make_synth_model
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), "vamd_models", "bench_spk_xvector_v1")
    if rank == 0 and not os.path.exists(os.path.join(cache, "README")):
        tmp = cache + f".tmp{os.getpid()}"
        make_synth_model.make_spk_model(tmp, **SPK_DIMS)
        os.rename(tmp, cache)
    if dist is not None:
        dist.barrier()
    return cache


def _spk_cpu_init(model):
    import oracle_xvector as OX
    from threadpoolctl import threadpool_limits
    _ORC["blas"] = threadpool_limits(1)  # one core per worker (the oracle's numpy GEMMs)
    _ORC["spk"] = OX.OracleSpk(model)


def _spk_cpu_job(w):
    t = time.time()
    _ORC["spk"].xvector(w, 0, [1] * 100000)
    return time.time() - t


def run_spk(args, dist, rank, world):
    """BASELINE config 5's speaker path per GPU: 1024 streams / 8 GPUs = 128
    utterances (10 s each, all frames selected) per step, extracted through
    vamd_spk_extract_batch (speaker MFCC, sliding CMN, the frame-level TDNN
    layers as one GEMM launch per layer over every utterance, statistics
    pooling, head, whitening; xvector.h).  The value is audio seconds per
    wall second over all ranks; the roofline is the frame-level layers'
    fp32 GEMM flops over their HIP-event time on the extractor's stream."""
    import ctypes as C
    import vosk
    from vosk import engine as ve
    vosk.SetLogLevel(-1)
    if ve.device_count() == 0:
        raise SystemExit("bench.py: no HIP device visible")
    model = spk_bench_model(rank, dist)
    spk = vosk.SpkModel(model)
    so = C.CDLL(os.path.join(os.path.dirname(vosk.__file__), "libvosk.so"))
    so.vamd_spk_extract_batch.restype = C.c_int
    so.vamd_spk_stats.restype = C.c_int
    n = 1024 // 8 if args.streams == 256 else args.streams
    secs = 10.0
    base = load_wave()
    waves = [np.ascontiguousarray(stream_audio(base, 20_000 + rank * n + i, int(secs * SR)), np.float32)
             for i in range(n)]
    keep = np.ones(int(secs * 100) // 3 + 8, np.int8)
    wp = (C.c_void_p * n)(*[w.ctypes.data for w in waves])
    kp = (C.c_void_p * n)(*([keep.ctypes.data] * n))
    ln = np.array([len(w) for w in waves], np.int64)
    rate = np.full(n, SR, np.int32)
    first = np.zeros(n, np.int32)
    nk = np.full(n, len(keep), np.int32)
    cap = 1024
    out = np.zeros((n, cap), np.float32)
    nf = np.zeros(n, np.int32)
    st = np.zeros(n, np.int32)

    def step():
        r = so.vamd_spk_extract_batch(C.c_void_p(spk._handle), n, wp, C.c_void_p(ln.ctypes.data),
                                      C.c_void_p(rate.ctypes.data), C.c_void_p(first.ctypes.data), kp,
                                      C.c_void_p(nk.ctypes.data), C.c_void_p(out.ctypes.data), cap,
                                      C.c_void_p(nf.ctypes.data), C.c_void_p(st.ctypes.data))
        if r != n or not (st > 0).all():
            raise SystemExit(f"bench.py spk: extraction failed ({r}, {int((st > 0).sum())} vectors)")

    def stats():
        b, u, fl, ms = C.c_longlong(0), C.c_longlong(0), C.c_double(0), C.c_double(0)
        so.vamd_spk_stats(C.c_void_p(spk._handle), C.byref(b), C.byref(u), C.byref(fl), C.byref(ms))
        return b.value, u.value, fl.value, ms.value

    steps = args.steps or 10
    for _ in range(args.warmup):
        step()
    b0, u0, fl0, ms0 = stats()
    if dist is not None:
        dist.barrier()
    t0 = time.time()
    for _ in range(steps):
        step()
    elapsed = _max_over_ranks(dist, time.time() - t0)
    b1, u1, fl1, ms1 = stats()
    audio = n * secs * steps * world
    flops, lms = fl1 - fl0, ms1 - ms0
    tf = flops / (lms * 1e-3) / 1e12 if lms > 0 else 0.0
    res = {
        "metric": "speaker x-vector extraction real-time factor (xRT), config 5 per-GPU share",
        "value": round(audio / elapsed, 2), "unit": "xRT", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic: test.wav tiled/perturbed per stream; random-init x-vector weights",
        "config": {"workload": "spk_xvector_batch", "utterances_per_gpu_step": n, "utterance_seconds": secs,
                   "model": "synthetic x-vector (tdnn 512 x4 -> 1500, stats pooling, embed 512, out 128)",
                   "parallelism": f"dp{world}"},
        "launch_sequences_per_step": (b1 - b0) / steps, "utterances_per_step": (u1 - u0) / steps,
        "roofline": {"bound": "mfma", "kernel": "nnet GEMMs of the frame-level layers",
                     "achieved": round(tf, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": tf / FP32_PEAK_TFLOPS, "traffic": None,
                     "layers_ms_per_step": round(lms / steps, 3),
                     "gflop_per_step": round(flops / steps / 1e9, 3)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import multiprocessing as mp
        workers = cpu_workers()
        sample = (waves * (1 + 8 * workers // n))[:8 * workers]
        with mp.get_context("fork").Pool(workers, initializer=_spk_cpu_init, initargs=(model,)) as pool:
            t = time.time()
            pool.map(_spk_cpu_job, sample, chunksize=1)
            wall = time.time() - t
        res["cpu_baseline"] = {
            "value": round(len(sample) * secs / wall, 3), "unit": "xRT", "cores": workers, "kind": "port",
            "sample": f"{len(sample)} of the step's utterances ({secs:.0f} s each) through the oracle "
                      f"(tests/oracle_xvector.py: numpy MFCC and frame layers, C CMN / pooling / head), "
                      f"{workers} worker processes with one BLAS thread each"}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()

if __name__ == "__main__":
    main()
