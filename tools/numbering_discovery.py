"""What does the static expansion's state numbering change on a lookahead
model, against OpenFST's lazy ComposeFst numbering the reference decodes
with (LookaheadComposeFst per recognizer, src/recognizer.cc:31-37;
src/model.cc:282-285)?

Kaldi's HashList buckets tokens by state id (state % hash_size), so the
Kaldi-order search depends on the numbering.  The reference's ids come from
OpenFST's lazy composition: the start is 0 and a state's arc destinations
take the next ids, in the composed arc order, when the decoder first expands
it (orc_dec_opts.lazy_*, oracle.c kd_expand).  libvosk decodes a static
expansion, trimmed to co-accessible states and renumbered breadth-first
(graph_compose.cc ConnectCanonical).  This decodes the same streams with the
Kaldi-order oracle three ways:

  A  the decoding graph libvosk builds (trimmed, breadth-first ids): the GPU's
     semantics, bit-identical to the GPU decoder
  B  the untrimmed composition in OpenFST's arc order, bucketed by lazy
     discovery ids: the reference's semantics (as far as the composition
     restatement is OpenFST's)
  C  the untrimmed composition with its expansion-order ids (no lazy
     numbering): separates the effect of the trim from that of the ids

and reports per pair the streams whose 1-best word sequence differs, the
word errors between them, and the frames whose token count differs.

usage: python tools/numbering_discovery.py [streams] [seconds] [out.json]
"""
import json
import multiprocessing as mp
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "vosk-api_amd", "tools"),
          os.path.join(REPO, "vosk-api_amd")):
    sys.path.insert(0, p)
import kaldi_formats as kf  # noqa: E402
import oracle_graph as OG  # noqa: E402
import oracle_py  # noqa: E402
import conftest  # noqa: E402
from conftest import perturbed_stream  # noqa: E402

_W = {}


def _init(canon, raw):
    _W["a"] = oracle_py.OracleModel(canon, fpc=51)
    _W["r"] = oracle_py.OracleModel(raw, fpc=51)
    g = kf.read_fst(os.path.join(raw, "graph", "HCLG.fst"))
    _W["lazy"] = (np.ascontiguousarray(g.row, np.int64), np.ascontiguousarray(g.nextstate, np.int32))


def _job(args):
    i, secs, base = args
    x = perturbed_stream(base, 6000 + i, seconds=secs)
    a, r = _W["a"], _W["r"]
    llh = a.loglikes(x)
    out = {}
    for name, o, lazy in (("A", a, None), ("B", r, _W["lazy"]), ("C", r, None)):
        d = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, True, kaldi=True, lazy=lazy)
        out[name] = (list(map(int, d["words"])), np.asarray(d["ntok"]).tolist(),
                     int((np.asarray(d["ntok"]) > o.max_active).sum()))
    return out


def wer(a, b):
    d = np.arange(len(b) + 1)
    for x in a:
        nd = d.copy()
        nd[0] = d[0] + 1
        for j, y in enumerate(b):
            nd[j + 1] = min(d[j + 1] + 1, nd[j] + 1, d[j] + (x != y))
        d = nd
    return int(d[-1])


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
    out_json = sys.argv[3] if len(sys.argv) > 3 else ""
    model = conftest._make_preset("la_small_en_us")
    canon = model.rstrip("/") + "_oracle_hclg"
    if not os.path.exists(os.path.join(canon, "graph", "lazy_ids.npz")):
        OG.expanded_hclg_model(model, canon + ".tmp")
        __import__("shutil").rmtree(canon, ignore_errors=True)
        os.rename(canon + ".tmp", canon)
    raw = model.rstrip("/") + "_oracle_raw"
    if not os.path.exists(os.path.join(raw, "graph", "HCLG.fst")):
        os.environ["VOSK_AMD_GRAPH_RAW"] = "1"
        _, nraw = OG.expanded_hclg_model(model, raw + ".tmp")
        del os.environ["VOSK_AMD_GRAPH_RAW"]
        os.rename(raw + ".tmp", raw)
    ga = kf.read_fst(os.path.join(canon, "graph", "HCLG.fst"))
    gr = kf.read_fst(os.path.join(raw, "graph", "HCLG.fst"))
    print(f"decoding graph: {len(ga.final)} states {len(ga.ilabel)} arcs; composition: {len(gr.final)} states "
          f"{len(gr.ilabel)} arcs", flush=True)
    base = conftest.np.frombuffer(__import__("wave").open(os.path.join(REPO, "tests", "golden", "test.wav"))
                                  .readframes(10 ** 7), "<i2").astype(np.float32)
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(workers, initializer=_init, initargs=(canon, raw)) as pool:
        res = pool.map(_job, [(i, secs, base) for i in range(n)], chunksize=1)
    rep = dict(streams=n, seconds=secs, graph_states=len(ga.final), composition_states=len(gr.final))
    words = sum(len(x["B"][0]) for x in res)
    rep["words_B"] = words
    rep["frames_over_max_active_B"] = sum(x["B"][2] for x in res)
    rep["frames"] = sum(len(x["B"][1]) for x in res)
    for p, q in (("A", "B"), ("C", "B"), ("A", "C")):
        diff = [i for i, x in enumerate(res) if x[p][0] != x[q][0]]
        errs = sum(wer(x[p][0], x[q][0]) for x in res)
        tokf = sum(int(np.sum(np.asarray(x[p][1]) != np.asarray(x[q][1]))) for x in res)
        rep[f"{p}_vs_{q}"] = dict(streams_1best_differ=len(diff), word_errors=errs,
                                  wer=round(errs / max(words, 1), 5), frames_token_count_differs=tokf,
                                  differing_streams=diff)
        print(f"{p} vs {q}: 1-best differs in {len(diff)} of {n} streams, {errs} word errors in {words} words, "
              f"token count differs in {tokf} of {rep['frames']} frames", flush=True)
    print(json.dumps(rep), flush=True)
    if out_json:
        with open(out_json, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
