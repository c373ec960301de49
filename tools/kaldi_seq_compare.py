#!/usr/bin/env python3
"""Order-independent token passing (what the GPU decoder and oracle.c's
orc_decode compute, bit-exactly) against the Kaldi-sequential restatement
(oracle.c orc_decode_kaldi: LatticeFasterDecoderTpl with its HashList order,
running emitting cutoff and LIFO epsilon queue) on the same log-likelihoods.

Reports per model: per-frame token-count differences, the 1-best word
sequence identity rate and word error rate between the two, and the relative
best-path cost difference.  Test infrastructure (CPU only).

usage: python tools/kaldi_seq_compare.py [--streams N] [--seconds S] [--json out.json] models...
  models: synth | wide | la_small_en_us | <model dir>
"""
import argparse
import json
import multiprocessing as mp
import os
import sys

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "vosk-api_amd"), os.path.join(REPO, "vosk-api_amd", "tools")):
    sys.path.insert(0, p)


def edit_distance(a, b):
    d = list(range(len(b) + 1))
    for i in range(1, len(a) + 1):
        prev, d[0] = d[0], i
        for j in range(1, len(b) + 1):
            cur = d[j]
            d[j] = min(d[j] + 1, d[j - 1] + 1, prev + (a[i - 1] != b[j - 1]))
            prev = cur
    return d[len(b)]


def model_dir(name):
    import conftest
    if name == "synth":
        return conftest._make("synth", seed=7, vocab=3000, num_pdfs=2000)
    if name == "wide":
        import shutil
        src = model_dir("synth")
        path = os.path.join(conftest.MODEL_CACHE, f"synth_wide_{conftest.SYNTH_VERSION}")
        if not os.path.exists(os.path.join(path, "README")):
            shutil.copytree(src, path + ".tmp")
            with open(os.path.join(path + ".tmp", "conf", "model.conf"), "a") as f:
                f.write("--beam=30.0\n--max-active=20000\n")
            os.rename(path + ".tmp", path)
        return path
    if name == "la_small_en_us":
        import make_synth_model
        import oracle_graph as OG
        path = os.path.join(conftest.MODEL_CACHE, "bench_la_small_en_us_v4")
        if not os.path.exists(os.path.join(path, "README")):
            make_synth_model.make_preset(name, path + ".tmp")
            os.rename(path + ".tmp", path)
        out = path + "_oracle_hclg"
        if not os.path.exists(os.path.join(out, "graph", "lazy_ids.npz")):
            OG.expanded_hclg_model(path, out + ".tmp")
            __import__("shutil").rmtree(out, ignore_errors=True)
            os.rename(out + ".tmp", out)
        return out
    return name


_M = {}


def _init(d):
    import oracle_py
    _M["o"] = oracle_py.OracleModel(d, fpc=51)


def _job(args):
    i, seconds = args
    import conftest
    import wave
    o = _M["o"]
    w = wave.open(os.path.join(REPO, "tests", "golden", "test.wav"), "rb")
    base = np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float32)
    x = conftest.perturbed_stream(base, 7000 + i, seconds=seconds)
    llh = o.loglikes(x)
    g = o.graph
    a = g.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, True)
    b = g.decode(llh, o.beam, o.max_active, o.min_active, o.beam_delta, True, kaldi=True)
    return dict(words_oi=a["words"], words_k=b["words"], cost_oi=a["best_cost"], cost_k=b["best_cost"],
                ntok_oi=a["ntok"].tolist(), ntok_k=b["ntok"].tolist(), max_active=o.max_active)


def compare(name, streams, seconds, workers):
    d = model_dir(name)
    with mp.get_context("fork").Pool(workers, initializer=_init, initargs=(d,)) as pool:
        res = pool.map(_job, [(i, seconds) for i in range(streams)], chunksize=1)
    same = sum(r["words_oi"] == r["words_k"] for r in res)
    errs = sum(edit_distance(r["words_k"], r["words_oi"]) for r in res)
    nwords = sum(len(r["words_k"]) for r in res)
    rel = [abs(r["cost_oi"] - r["cost_k"]) / max(abs(r["cost_k"]), 1e-9) for r in res]
    dt = np.concatenate([np.array(r["ntok_k"]) - np.array(r["ntok_oi"]) for r in res])
    nk = np.concatenate([np.array(r["ntok_k"]) for r in res])
    frac_equal = float((dt == 0).mean())
    return {"model": name, "streams": streams, "seconds": seconds, "frames": int(dt.size),
            "one_best_identical": same / streams, "wer_oi_vs_kaldi": errs / max(nwords, 1),
            "kaldi_words": nwords, "rel_cost_delta_max": max(rel), "rel_cost_delta_mean": float(np.mean(rel)),
            "oi_cost_lower_or_equal": sum(r["cost_oi"] <= r["cost_k"] + 1e-6 for r in res) / streams,
            "frames_with_equal_token_count": frac_equal,
            "token_delta_p50": float(np.percentile(dt, 50)), "token_delta_p1": float(np.percentile(dt, 1)),
            "token_delta_p99": float(np.percentile(dt, 99)),
            "rel_token_delta_mean": float(np.mean(np.abs(dt) / np.maximum(nk, 1))),
            "frames_over_max_active": float((nk > res[0]["max_active"]).mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("models", nargs="*", default=["synth", "wide", "la_small_en_us"])
    ap.add_argument("--streams", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--workers", type=int, default=min(8, len(os.sched_getaffinity(0))))
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = [compare(m, a.streams, a.seconds, a.workers) for m in a.models]
    for r in out:
        print(json.dumps(r))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
