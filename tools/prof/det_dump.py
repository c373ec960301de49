"""Dump bench-model segment lattices (Kaldi-order oracle, pruned as the GPU
hands them over) for tools/prof/det_prof.cc (host result-chain profiling).
usage: python tools/prof/det_dump.py out.bin [streams] [seconds]"""
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "vosk-api_amd"),
                os.path.join(REPO, "vosk-api_amd", "tools")]
import numpy as np  # noqa: E402


def main():
    out, n, secs = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8, float(sys.argv[3]) if len(sys.argv) > 3 else 6.25
    import bench
    import oracle_lattice as OL
    import oracle_py
    model = bench.bench_model(0, None, "la_small_en_us")
    o = oracle_py.OracleModel(bench.oracle_model_dir(model), fpc=51)
    base = bench.load_wave()
    ty, fi, lo = OL.align_tables(o.tm, os.path.join(o.dir, "graph", "phones", "word_boundary.int"))
    tf = OL.tid_first(o.tm)
    with open(out, "wb") as f:
        def arr(a, dt):
            a = np.ascontiguousarray(a, dt)
            f.write(struct.pack("<q", a.size))
            f.write(a.tobytes())
        arr(o.graph.ilabel, np.int32); arr(o.graph.olabel, np.int32)
        arr(o.tm.tid2phone, np.int32); arr(tf, np.int8)
        arr(ty, np.int8); arr(fi, np.int8); arr(lo, np.int8)
        f.write(struct.pack("<q", n))
        for i in range(n):
            x = bench.stream_audio(base, 10_000 + i, int(secs * bench.SR))
            r = o.graph.decode(o.loglikes(x), o.beam, o.max_active, o.min_active, o.beam_delta, True,
                               lattice=True, kaldi=True)
            L = OL.prune(OL.raw_from_oracle(r, o.graph, True), 6.0)
            f.write(struct.pack("<q", int(L["num_frames"])))
            for k, dt in (("frame_begin", np.int32), ("tok_state", np.int32), ("tok_cost", np.float32),
                          ("link_src", np.int32), ("link_dst", np.int32), ("link_arc", np.int32),
                          ("link_graph", np.float32), ("link_ac", np.float32), ("final_cost", np.float32)):
                arr(L[k], dt)
            print(i, len(L["link_src"]), flush=True)


if __name__ == "__main__":
    main()
