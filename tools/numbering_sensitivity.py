"""How much does Kaldi's HashList order -- which depends on state ids
(bucket = state % hash_size) -- move the 1-best of the Kaldi-order decoder?

The reference numbers the states of a lookahead model's composed graph
lazily, per recognizer, in discovery order (LookaheadComposeFst,
src/recognizer.cc:31-37); libvosk numbers its static expansion breadth-first
(DESIGN.md §4).  This measures the effect of numbering alone: the oracle's
Kaldi-order decoder (orc_decode_kaldi) on the bench model's expanded graph
and on copies whose state ids are randomly permuted (same arcs, same arc
order), over the same streams.  Prints per numbering: streams whose 1-best
word sequence differs from the original numbering's, word errors between
them, frames with a different token count.

usage: python tools/numbering_sensitivity.py [model_dir] [streams] [seconds]
"""
import json
import multiprocessing as mp
import os
import shutil
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "vosk-api_amd", "tools"), os.path.join(REPO, "vosk-api_amd")):
    sys.path.insert(0, p)
import kaldi_formats as kf  # noqa: E402
import oracle_py  # noqa: E402
from conftest import perturbed_stream  # noqa: E402

_W = {}


def permuted_model(src, dst, seed):
    g = kf.read_fst(os.path.join(src, "graph", "HCLG.fst"))
    S = len(g.final)
    rng = np.random.default_rng(seed)
    perm = rng.permutation(S).astype(np.int64)  # old -> new
    inv = np.argsort(perm)                       # new -> old
    deg = (g.row[1:] - g.row[:-1])[inv]
    row = np.zeros(S + 1, np.int64)
    row[1:] = np.cumsum(deg)
    idx = np.concatenate([np.arange(g.row[o], g.row[o + 1]) for o in inv]) if S else np.zeros(0, np.int64)
    h = kf.Fst(int(perm[g.start]), g.final[inv].copy(), row, g.ilabel[idx].copy(), g.olabel[idx].copy(),
               g.weight[idx].copy(), perm[g.nextstate[idx]].astype(np.int32))
    if os.path.exists(dst):
        shutil.rmtree(dst)
    shutil.copytree(src, dst, ignore=shutil.ignore_patterns("HCLG.fst"))
    kf.write_const_fst(os.path.join(dst, "graph", "HCLG.fst"), h)
    return dst


def _init(dirs):
    _W["o"] = [oracle_py.OracleModel(d, fpc=51) for d in dirs]


def _job(args):
    i, secs, base = args
    x = perturbed_stream(base, 6000 + i, seconds=secs)
    o0 = _W["o"][0]
    llh = o0.loglikes(x)
    out = []
    for o in _W["o"]:
        r = o.graph.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, True, kaldi=True)
        out.append((list(map(int, r["words"])), np.asarray(r["ntok"]).tolist()))
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
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.environ.get("TMPDIR", "/tmp"), "vamd_models",
                                                                 "bench_la_small_en_us_v4_oracle_hclg")
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    secs = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0
    dirs = [src] + [permuted_model(src, src.rstrip("/") + f"_perm{k}", 100 + k) for k in range(2)]
    import bench
    base = bench.load_wave()
    with mp.get_context("fork").Pool(min(16, os.cpu_count() or 1), initializer=_init, initargs=(dirs,)) as pool:
        res = pool.map(_job, [(i, secs, base) for i in range(n)], chunksize=1)
    rep = {"model": src, "streams": n, "seconds": secs, "numberings": {}}
    for k in range(1, len(dirs)):
        diff = sum(1 for r in res if r[0][0] != r[k][0])
        errs = sum(wer(r[0][0], r[k][0]) for r in res)
        words = sum(len(r[0][0]) for r in res)
        fr = sum(len(r[0][1]) for r in res)
        frd = sum(int(np.sum(np.asarray(r[0][1]) != np.asarray(r[k][1]))) for r in res)
        rep["numberings"][f"random_permutation_{k}"] = {
            "streams_with_different_1best": diff, "word_errors": errs, "words": words,
            "wer_pct": round(100.0 * errs / max(words, 1), 3),
            "frames_with_different_token_count_pct": round(100.0 * frd / max(fr, 1), 3)}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
