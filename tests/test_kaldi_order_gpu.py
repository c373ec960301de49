"""Kaldi-order token passing on the GPU (the decoder's default)
against the Kaldi-sequential restatement of the reference decoder
(oracle.c orc_decode_kaldi: LatticeFasterDecoderTpl with its HashList order,
running emitting cutoff and LIFO epsilon queue; src/recognizer.cc:39-43,
src/batch_model.cc:78-80), on the GPU's own log-likelihoods: per-frame token
counts, best costs, cutoffs and the 1-best path bit-identical for 64 streams
decoded together, with max-active engaged, on

* the flat synthetic model (random nnet: flat scores, thousands of tokens),
  max-active lowered to 1500 so it binds in most frames, and
* the vosk-model-small-en-us-scale lookahead model (275 k-state expansion,
  beam 13 / max-active 7000).

The order-independent form (VOSK_AMD_DEC_ORDER=parallel) stays available and
is checked against orc_decode on the same streams."""
import multiprocessing as mp
import os
import shutil

import numpy as np
import pytest

import oracle_py
from conftest import perturbed_stream

pytestmark = pytest.mark.gpu

NSTREAMS = 64
_ORC = {}


def _orc_job(i):
    o = _ORC["o"]
    r = o.graph.decode(_ORC["llh"][i], o.beam, o.max_active, o.min_active, o.beam_delta, True,
                       kaldi=_ORC["kaldi"], lazy=_ORC["lazy"])
    return dict(ntok=r["ntok"], best=r["best"], cutoff=r["cutoff"], next_cutoff=r["next_cutoff"],
                path=r["path"], cost=r["best_cost"])


def _oracle(oracle_dir, llhs, kaldi=True, lazy=None):
    o = oracle_py.OracleModel(oracle_dir, fpc=51)
    _ORC.update(o=o, llh=llhs, kaldi=kaldi, lazy=lazy)
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(workers) as pool:
        res = pool.map(_orc_job, range(len(llhs)), chunksize=1)
    _ORC.clear()
    return res, o.max_active


def _gpu(model_dir, waves):
    from vosk import engine
    e = engine.Engine(model_dir, frames_per_chunk=51, max_streams=len(waves), stats=True, keep_llh=True)
    ss = [e.new_stream() for _ in waves]
    for s, w in zip(ss, waves):
        e.accept(s, w, finished=True)
    e.advance(ss)
    out = []
    for s in ss:
        st = e.decoder_state(s)
        assert st["err"] == 0, st
        out.append(dict(stats=e.stats(s), llh=e.llh(s), path=e.best_path(s, use_final=True)))
    e.close()
    return out


def _compare(gpu, ref, max_active):
    over = 0
    for k, (g, r) in enumerate(zip(gpu, ref)):
        st = g["stats"]
        d = np.nonzero(st[:, 1].astype(np.int64) != r["ntok"][1:len(st) + 1])[0]
        if len(d):
            f = int(d[0])
            print(f"stream {k}: first token-count difference at frame {f}: gpu {st[max(f - 2, 0):f + 3, 1]} "
                  f"oracle {r['ntok'][max(f - 2, 0) + 1:f + 4]} cutoff gpu {st[f, 5]} oracle {r['cutoff'][f]} "
                  f"next {st[f, 6]} / {r['next_cutoff'][f]} best {st[f, 4]} / {r['best'][f + 1]} in {st[f, 0]}")
        np.testing.assert_array_equal(st[:, 1].astype(np.int64), r["ntok"][1:], err_msg=f"stream {k} tokens")
        np.testing.assert_array_equal(st[:, 4], r["best"][1:], err_msg=f"stream {k} best costs")
        np.testing.assert_array_equal(st[:, 5], r["cutoff"], err_msg=f"stream {k} cutoffs")
        np.testing.assert_array_equal(st[:, 6], r["next_cutoff"], err_msg=f"stream {k} next cutoffs")
        arcs, cost, _ = g["path"]
        np.testing.assert_array_equal(arcs, r["path"], err_msg=f"stream {k} 1-best")
        assert cost == pytest.approx(r["cost"], abs=1e-6)
        over += int((st[:, 0] > max_active).sum())
    assert over > 0  # max-active engaged


@pytest.fixture(scope="module")
def flat_model(synth_model, tmp_path_factory):
    d = str(tmp_path_factory.mktemp("flat") / "m")
    shutil.copytree(synth_model, d, symlinks=True)
    with open(os.path.join(d, "conf", "model.conf"), "a") as f:
        f.write("--max-active=1500\n")
    return d


def test_flat_model_64_streams(flat_model, test_wave, monkeypatch):
    monkeypatch.delenv("VOSK_AMD_DEC_ORDER", raising=False)
    waves = [perturbed_stream(test_wave, 4000 + i, seconds=4.0 + 0.05 * i) for i in range(NSTREAMS)]
    gpu = _gpu(flat_model, waves)
    ref, max_active = _oracle(flat_model, [g["llh"] for g in gpu])
    assert max_active == 1500
    _compare(gpu, ref, max_active)


def test_lookahead_model_64_streams(synth_la_small_en_us, test_wave, monkeypatch):
    """The same with the static graph's own ids (VOSK_AMD_LAZY_IDS=0)."""
    import oracle_graph as OG
    monkeypatch.delenv("VOSK_AMD_DEC_ORDER", raising=False)
    monkeypatch.setenv("VOSK_AMD_LAZY_IDS", "0")
    waves = [perturbed_stream(test_wave, 5000 + i, seconds=4.0 + 0.05 * i) for i in range(NSTREAMS)]
    gpu = _gpu(synth_la_small_en_us, waves)
    out = synth_la_small_en_us.rstrip("/") + "_oracle_hclg"
    if not os.path.exists(os.path.join(out, "graph", "lazy_ids.npz")):
        OG.expanded_hclg_model(synth_la_small_en_us, out + ".tmp")
        __import__("shutil").rmtree(out, ignore_errors=True)
        os.rename(out + ".tmp", out)
    ref, max_active = _oracle(out, [g["llh"] for g in gpu])
    _compare(gpu, ref, max_active)


def test_lookahead_model_lazy_numbering_64_streams(synth_la_small_en_us, test_wave, monkeypatch):
    """OpenFST's lazy ComposeFst numbering (src/recognizer.cc:31-37):
    the GPU buckets its HashList by the ids OpenFST would give the composed
    states as the decoder expands them (libvosk's lazy CSR, vamd_graph_lazy);
    the oracle decodes the same graph with the same CSR (oracle.c kd_expand;
    that this equals decoding the untrimmed composition in its own arc order
    is tests/test_lazy_numbering.py)."""
    import oracle_graph as OG
    monkeypatch.delenv("VOSK_AMD_DEC_ORDER", raising=False)
    monkeypatch.delenv("VOSK_AMD_LAZY_IDS", raising=False)
    waves = [perturbed_stream(test_wave, 5000 + i, seconds=4.0 + 0.05 * i) for i in range(NSTREAMS)]
    gpu = _gpu(synth_la_small_en_us, waves)
    out = synth_la_small_en_us.rstrip("/") + "_oracle_hclg"
    if not os.path.exists(os.path.join(out, "graph", "lazy_ids.npz")):
        OG.expanded_hclg_model(synth_la_small_en_us, out + ".tmp")
        __import__("shutil").rmtree(out, ignore_errors=True)
        os.rename(out + ".tmp", out)
    row, nxt, ids = OG.lazy_csr(synth_la_small_en_us)
    assert ids > 0
    ref, max_active = _oracle(out, [g["llh"] for g in gpu], lazy=(row, nxt))
    _compare(gpu, ref, max_active)


def test_parallel_form_stays_available(flat_model, test_wave, monkeypatch):
    """VOSK_AMD_DEC_ORDER=parallel: the order-independent form, bit-exact
    against orc_decode."""
    monkeypatch.setenv("VOSK_AMD_DEC_ORDER", "parallel")
    waves = [perturbed_stream(test_wave, 4000 + i, seconds=3.0) for i in range(8)]
    gpu = _gpu(flat_model, waves)
    ref, max_active = _oracle(flat_model, [g["llh"] for g in gpu], kaldi=False)
    _compare(gpu, ref, max_active)
