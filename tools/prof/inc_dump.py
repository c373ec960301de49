"""Dump one bench-model stream's decoder records (Kaldi-order oracle) and the
AdvanceDecoding ends of 0.25-s calls for tools/prof/inc_prof.cc (host
profiling of the KaldiRecognizer's incremental lattice).
usage: python tools/prof/inc_dump.py out.bin [seconds]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "vosk-api_amd")]
import numpy as np  # noqa: E402


def main():
    out = sys.argv[1]
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    import bench
    import oracle_incremental as OI
    import oracle_lattice as OL
    import oracle_py
    model = bench.bench_model(0, None, "la_small_en_us")
    o = oracle_py.OracleModel(bench.oracle_model_dir(model))
    x = bench.stream_audio(bench.load_wave(), 900, int(secs * bench.SR))
    r = o.graph.decode(o.loglikes(x), o.beam, o.max_active, o.min_active, o.beam_delta, True,
                       lattice=True, kaldi=True)
    frames = OI.frames_from_oracle(r, o.graph)
    g = o.graph
    with open(out, "wb") as f:
        def w(a, dt):
            a = np.ascontiguousarray(a, dt)
            f.write(np.int64(a.size).tobytes())
            f.write(a.tobytes())
        w(g.ilabel, np.int32); w(g.olabel, np.int32); w(g.weight, np.float32); w(g.final, np.float32)
        w([g.start], np.int32)
        w(o.tm.tid2phone, np.int32); w(OL.tid_first(o.tm).astype(np.int8), np.int8)
        w([len(frames)], np.int32)
        for st, co, links, off in frames:
            w(st, np.int32); w(co, np.float32); w([off], np.float32)
            w(np.array([(a, b, c) for a, b, c, _ in links], np.int32).reshape(-1, 3), np.int32)
            w([x[3] for x in links], np.float32)
        # AdvanceDecoding ends of 0.25-s calls (7-9 frames each), then the final lattice
        ends, d = [], 0
        while d < len(frames) - 1:
            d = min(d + 8, len(frames) - 1)
            ends.append(d)
        w([0] * len(ends) + [2], np.int32); w(ends + [0], np.int32)
    print(len(frames), "frames,", sum(len(fr[2]) for fr in frames), "links")


if __name__ == "__main__":
    main()
