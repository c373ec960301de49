"""Host result-chain timing (CPU only): the Kaldi-order oracle decodes
synthetic bench streams on the bench model's expanded graph with lattices,
and libvosk's result chain (prune, pruned phone + word determinization,
graph scale, word alignment, MBR) runs over each lattice with its stage
timings.  usage: python tools/det_bench.py [--streams N] [--seconds S] [--reps R]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "vosk-api_amd"),
                os.path.join(REPO, "vosk-api_amd", "tools")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=6.25)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import bench
    import oracle_lattice as OL
    import oracle_py
    from vosk import engine
    model = bench.bench_model(0, None, "la_small_en_us")
    o = oracle_py.OracleModel(bench.oracle_model_dir(model), fpc=51)
    base = bench.load_wave()
    engine.set_phones(o.tm.tid2phone, OL.tid_first(o.tm))
    tables = OL.align_tables(o.tm, os.path.join(o.dir, "graph", "phones", "word_boundary.int"))
    rows = []
    for i in range(a.streams):
        x = bench.stream_audio(base, 10_000 + i, int(a.seconds * bench.SR))
        r = o.graph.decode(o.loglikes(x), o.beam, o.max_active, o.min_active, o.beam_delta, True,
                           lattice=True, kaldi=True)
        # the GPU decoder hands over lattices already pruned to the lattice
        # beam (PruneActiveTokens in the kernel, prune_final_kernel): the
        # oracle's raw lattice pruned the same way first
        L = OL.prune(OL.raw_from_oracle(r, o.graph, True), 6.0)
        best = None
        for _ in range(a.reps):
            t = time.perf_counter()
            got = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, 0.9, 0, align=tables,
                                       timings=True)
            ms = (time.perf_counter() - t) * 1e3
            if best is None or ms < best[0]:
                best = (ms, got.get("ms"))
        rows.append({"links": int(len(L["link_src"])), "frames": int(L["num_frames"]), "wall_ms": round(best[0], 3),
                     "stages_ms": best[1]})
        print(json.dumps(rows[-1]), flush=True)
    tot = sum(r["wall_ms"] for r in rows)
    out = {"streams": a.streams, "seconds": a.seconds, "mean_ms_per_segment": round(tot / len(rows), 3),
           "rows": rows}
    print(json.dumps({k: v for k, v in out.items() if k != "rows"}))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
