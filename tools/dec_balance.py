"""Per-stream decoder balance on the engine bench workload: per-stream phase
clocks vs tokens created, pipelined and in-order.  Development tool."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["VOSK_AMD_DEC_PROFILE"] = "1"
import bench  # noqa: E402


def run(model, base, S, pipe, steps=12):
    from vosk import engine as ve
    e = ve.Engine(model, frames_per_chunk=51, max_streams=S, stats=True, time_kernels=True, pipeline=pipe,
                  lattice=True)
    chunk = e.fpc * 160
    e.set_step_samples(chunk)
    ss = []
    for i in range(S):
        s = e.new_stream()
        e.preload(s, bench.stream_audio(base, i, (steps + 4) * chunk), finished=False)
        ss.append(s)
    for _ in range(steps):
        e.step(ss)
    st = e.stage_times()
    per = e.decoder_phases_per_stream()[:S]
    clk = per[:, e.PHASE_CLOCK_IDX].sum(1).astype(np.float64)
    created = per[:, 12].astype(np.float64)
    heavy = int(np.argmax(clk))
    frames = max(int(per[heavy, 15]), 1)
    mean_frames = max(float(per[:, 15].mean()), 1.0)
    phases = {e.PHASES[i]: (round(per[heavy, i] / frames), round(float(per[:, i].mean()) / mean_frames))
              for i in range(len(e.PHASES)) if e.PHASES[i] not in ("-", "frames")}
    e.close()
    return {"heavy_vs_mean_per_frame": phases, "pipeline": pipe, "streams": S, "decode_ms_per_launch": st["decode"][0] / max(st["decode"][1], 1),
            "clk_mean": clk.mean(), "clk_max_over_mean": clk.max() / clk.mean(),
            "created_max_over_mean": created.max() / created.mean(),
            "corr_clk_created": float(np.corrcoef(clk, created)[0, 1]),
            "clk_per_created_cv": float((clk / created).std() / (clk / created).mean()),
            "clk_per_launch_max_ms_at_2.4GHz": clk.max() / steps / 2.4e6}


def main():
    model = bench.bench_model(0, None, "la_small_en_us")
    import vosk
    vosk.SetLogLevel(-1)
    base = bench.load_wave()
    for S, pipe in ((256, False),):
        print(json.dumps(run(model, base, S, pipe)), flush=True)


if __name__ == "__main__":
    main()
