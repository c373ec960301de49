#!/usr/bin/env python3
"""Aggregate real-time factor of the Vosk hot path on MI355X.

Workload (BASELINE.json configs[2], the largest single-GPU configuration):
BatchRecognizer-style decoding of 256 concurrent synthetic 16 kHz streams per
GPU through libvosk.so's GPU engine -- MFCC -> looped TDNN-F nnet3 (fp32 MFMA)
-> token-passing beam search (beam 13, max-active 7000) -- with the
frames_per_chunk = 51 chunking of src/batch_model.cc:84-88.  A "step" is one
engine pass that advances every stream by one 8160-sample chunk (0.51 s of
audio); stream audio is resident in HBM before the timed region (per-step
PCIe traffic is excluded; see DESIGN.md for the host-fed rate).

Model: no Vosk model is available offline, so a seeded synthetic model with
the reference recipe's TDNN-F topology (training/local/chain/run_tdnn.sh:
98-129, random-init weights, BatchNorm calibrated on test.wav) and a 20k-word
lexicon-tree HCLG is generated in the real Kaldi/OpenFST formats.  Streams
are test.wav tiled, shifted, gained and noised per BASELINE.md.

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


def load_wave():
    w = wave.open(os.path.join(REPO, "tests", "golden", "test.wav"), "rb")
    return np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)


def stream_audio(base, i, n):
    from conftest import perturbed_stream
    return perturbed_stream(base, i, seconds=n / SR)


def bench_model(rank, dist):
    import make_synth_model
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), "vamd_models", "bench_v3")
    if rank == 0 and not os.path.exists(os.path.join(cache, "README")):
        make_synth_model.make_model(cache, seed=11, vocab=20000, num_pdfs=2000)
    if dist is not None:
        dist.barrier()
    return cache


def cpu_baseline(model, base, streams, seconds, workers):
    """Oracle (single-threaded C restatement) timed on host cores: one stream
    per worker process at a time (the transcribe_scp.py Pool pattern)."""
    import multiprocessing as mp
    jobs = [(model, i, seconds) for i in range(streams)]
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
    _ORC["m"] = oracle_py.OracleModel(model, fpc=51)  # the engine's chunking (i-vector per chunk)
    _ORC["base"] = load_wave()


def _cpu_job(args):
    model, i, seconds = args
    x = stream_audio(_ORC["base"], 10_000 + i, int(seconds * SR))
    t = time.time()
    _ORC["m"].recognize(x)
    return len(x) / SR, time.time() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--streams", type=int, default=256, help="streams per GPU")
    ap.add_argument("--model", default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="decoder in order after the nnet (default: decoder of step i-1 "
                         "concurrently with the nnet of step i on a second HIP stream)")
    ap.add_argument("--no-lattice", action="store_true",
                    help="decoder without lattice links (default: Kaldi forward links kept in "
                         "HBM per stream, as the reference's batch decoder produces lattices)")
    ap.add_argument("--workload", choices=("static", "dynamic"), default="static",
                    help="static (default, the headline): S equal-length streams per GPU, HBM "
                         "resident; dynamic: a node-wide queue of variable-length utterances "
                         "admitted per epoch to the GPUs with the most free slots (one int32 "
                         "all-gather per epoch, vosk/shard.py)")
    ap.add_argument("--no-single-stream", action="store_true",
                    help="skip the single-stream accept_waveform latency measurement")
    ap.add_argument("--cpu-streams", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=300.0)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    os.environ["VOSK_AMD_DEVICE"] = str(local_rank)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        tdist.init_process_group(backend=backend)
        dist = tdist

    model = args.model or bench_model(rank, dist)
    import vosk
    from vosk import engine as ve
    vosk.SetLogLevel(-1)
    if ve.device_count() == 0:
        raise SystemExit("bench.py: no HIP device visible")
    S = args.streams
    if args.workload == "dynamic":
        return run_dynamic(args, model, dist, rank, world, local_rank)
    pipe = not args.no_pipeline
    e = ve.Engine(model, frames_per_chunk=51, max_streams=S, stats=True, time_kernels=True,
                  pipeline=pipe, lattice=not args.no_lattice)
    chunk = e.fpc * 160
    e.set_step_samples(chunk)
    base = load_wave()
    total_steps = args.warmup + args.steps + 2
    streams = []
    for i in range(S):
        s = e.new_stream()
        e.preload(s, stream_audio(base, rank * S + i, total_steps * chunk), finished=False)
        streams.append(s)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        e.step(streams)
    e.stage_times(reset=True)
    lat = []
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        e.step(streams)  # synchronises the engine stream before returning
        lat.append(time.perf_counter() - ts)
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        import torch
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    audio_s = args.steps * S * chunk / SR * world
    xrt = audio_s / elapsed

    st = e.stage_times()
    tot = e.decoder_totals()
    errs = sum(1 for s in streams if e.error(s))
    # decoder roofline: algorithmic bytes per launch:
    # 16*T_in + 16*E + 8*E + 16*T_new + 20*L, L = T_new backpointer links,
    # plus 16 B per lattice link record kept in HBM
    E = tot["arcs_emit"] + tot["arcs_eps"]
    dec_bytes = (16 * tot["tok_in"] + 24 * E + 16 * tot["tok_out"] + 20 * tot["tok_out"]
                 + 16 * tot.get("links", 0))
    dec_ms, dec_n = st["decode"]
    nnet_ms, nnet_n = st["nnet"]
    front_ms, front_n = st["front"]
    dec_launch_ms = dec_ms / max(dec_n, 1)
    dec_gbs = (dec_bytes / max(dec_n, 1)) / (dec_launch_ms * 1e-3) / 1e9 if dec_n else 0.0
    nnet_flops = e.flops_per_chunk * S * args.steps
    nnet_tflops = nnet_flops / (nnet_ms * 1e-3) / 1e12 if nnet_ms else 0.0
    # dominant kernel (rocprofv3 --stats: decode_kernel, one launch per step,
    # the largest share of GPU time): HBM roofline on algorithmic bytes, with
    # the measured HBM traffic per launch from the committed PMC summary
    traffic = None
    pmc_path = os.path.join(REPO, "profiles", "r01_decode_pmc.json")
    if os.path.exists(pmc_path):
        try:
            traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "kernel": "decode_kernel", "achieved": round(dec_gbs, 3),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": dec_gbs / HBM_PEAK_GBS,
                "traffic": traffic, "avg_launch_ms": round(dec_launch_ms, 4),
                "alg_bytes_per_launch": dec_bytes / max(dec_n, 1)}
    roofline_nnet = {"bound": "mfma", "kernel": "nnet GEMM launches (29 per step)",
                     "achieved": round(nnet_tflops, 4), "peak": FP32_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": nnet_tflops / FP32_PEAK_TFLOPS}

    # single-stream latency (BASELINE config 2): wall time of one
    # vosk_recognizer_accept_waveform call on a 0.25 s (8000-byte) chunk
    # through the public API, test_simple.py's feeding pattern, 30 s of audio
    single = None
    if rank == 0 and world == 1 and not args.no_single_stream:
        single = single_stream_latency(model, base)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        workers = min(16, os.cpu_count() or 1)
        v, a, w = cpu_baseline(model, base, args.cpu_streams, args.cpu_seconds, workers)
        cpu = {"value": round(v, 3), "unit": "xRT", "cores": workers, "kind": "port",
               "sample": f"{args.cpu_streams} synthetic streams x {args.cpu_seconds:.0f} s through "
                         f"the C oracle (MFCC + nnet3 + token passing), {workers} worker processes, "
                         f"{a:.0f} s audio in {w:.1f} s wall"}

    if rank == 0:
        lat_ms = np.array(lat) * 1e3
        if pipe:  # a chunk's nnet runs in one step, its decoding in the next
            lat_ms = lat_ms[1:] + lat_ms[:-1]
        out = {
            "metric": "aggregate real-time factor (xRT) + p50 per-chunk latency, vosk-model-small-en-us",
            "value": round(xrt, 2), "unit": "xRT", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic: test.wav tiled/shifted/gain/noise per BASELINE.md; seeded "
                    "random-init synthetic model (recipe TDNN-F topology, 20k-word HCLG)",
            "config": {"workload": "config3: BatchRecognizer-equivalent, 256 streams/GPU, "
                                   "GPU MFCC + nnet3 + WFST beam search, 1xMI355X per rank",
                       "streams_per_gpu": S, "global_streams": S * world,
                       "chunk_samples": chunk, "frames_per_chunk": e.fpc,
                       "beam": 13.0, "max_active": 7000, "parallelism": f"dp{world}",
                       "pipeline": "decoder(step i-1) || mfcc+nnet(step i), 2 HIP streams"
                                   if pipe else "in-order"},
            "p50_chunk_latency_ms": round(float(np.percentile(lat_ms, 50)), 3),
            "p90_chunk_latency_ms": round(float(np.percentile(lat_ms, 90)), 3),
            "p99_chunk_latency_ms": round(float(np.percentile(lat_ms, 99)), 3),
            "roofline": roofline,
            "roofline_nnet": roofline_nnet,
            "stages_ms_per_step": {"front": round(front_ms / args.steps, 4),
                                   "nnet": round(nnet_ms / args.steps, 4),
                                   "decode": round(dec_ms / args.steps, 4),
                                   "gpu_step": round(st["step"][0] / args.steps, 4)},
            "nnet_tflops": round(nnet_tflops, 4),
            "decoder": {"frames": tot["frames"],
                        "tokens_per_frame": round(tot["tok_out"] / max(tot["frames"], 1), 1),
                        "arcs_per_frame": round(E / max(tot["frames"], 1), 1),
                        "lattice_links_per_frame": round(tot.get("links", 0) / max(tot["frames"], 1), 1),
                        "stream_errors": errs},
            "cpu_baseline": cpu,
            "single_stream": single,
        }
        if os.environ.get("VOSK_AMD_DEC_PROFILE"):
            ph = e.decoder_phases()
            out["decoder_phase_clocks_per_frame"] = {
                k: round(v / max(ph["frames"], 1), 1) for k, v in ph.items() if k != "frames"}
            out["decoder_phase_clocks_per_frame"]["total"] = round(
                sum(ph[k] for k in e.PHASE_CLOCKS) / max(ph["frames"], 1), 1)
            # per-stream spread: the slowest stream sets each launch's time
            per = e.decoder_phases_per_stream()[:S]
            clk = per[:, e.PHASE_CLOCK_IDX].sum(1).astype(np.float64)
            out["decoder_stream_clocks"] = {
                "mean": round(float(clk.mean()), 1), "p50": round(float(np.percentile(clk, 50)), 1),
                "p90": round(float(np.percentile(clk, 90)), 1), "max": round(float(clk.max()), 1),
                "max_over_mean": round(float(clk.max() / max(clk.mean(), 1.0)), 3)}
        print(json.dumps(out), flush=True)
    e.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def single_stream_latency(model, base, seconds=30.0, chunk_bytes=8000):
    """One KaldiRecognizer (silence-weighted i-vectors, lattice results)
    fed 8000-byte chunks; p50/p90/p99 of the accept_waveform wall time, the
    stream's real-time factor, and a final result call's time."""
    import vosk
    x = stream_audio(base, 777, int(seconds * SR))
    data = np.clip(x, -32768, 32767).astype("<i2").tobytes()
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


def run_dynamic(args, model, dist, rank, world, local_rank):
    """Variable-length utterances (5-60 s, seeded) from one node-wide queue
    (3 x streams x GPUs of them), admitted every 4 steps to the ranks with the
    most free slots; a finished stream frees its slot.  Samples are uploaded
    when a stream is admitted (inside the timed region: this mode measures
    the admission path, not the headline)."""
    import vosk
    from vosk import engine as ve
    from vosk.shard import AdmissionController
    S = args.streams
    e = ve.Engine(model, frames_per_chunk=51, max_streams=S, stats=True, lattice=not args.no_lattice)
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
    # the utterances' samples exist before the timed region (host memory);
    # admission uploads them to the stream's HBM buffer
    wav = {}

    def utt(u):
        if u not in wav:
            wav[u] = stream_audio(base, 50_000 + u, int(lens[u]))
        return wav[u]
    for u in range(U):
        utt(u)
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
                x = utt(u)
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
        t = torch.tensor([elapsed, audio], dtype=torch.float64, device=dev)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        a = torch.tensor([audio], dtype=torch.float64, device=dev)
        dist.all_reduce(a, op=dist.ReduceOp.SUM)
        elapsed, tot_audio = float(t[0].item()), float(a.item())
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


if __name__ == "__main__":
    main()
