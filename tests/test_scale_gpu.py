"""BASELINE configs 3 and 4 at their stated per-GPU scale (256 streams).

* Config 3: 256 ``BatchRecognizer``s through ``vosk_batch_*`` (the
  reference's ``test_gpu_batch.py`` loop: 8000-byte feeds, ``Wait``,
  ``Result`` per round, ``FinishStream`` at each stream's end) on the
  vosk-model-small-en-us-scale lookahead bench model, 10-25 s streams (every
  eighth stream is long enough for the 20 s rule to end a segment).  Every
  result message -- segment boundaries, MBR words and word times -- equals the
  oracle's over the same stream: the batch segmentation restated per chunk
  (``oracle_endpoint.batch_segments_fast``), then the lattice of each segment
  through the Python result chain (``oracle_lattice.results``).
  Reference: src/batch_model.cc:23-121, src/batch_recognizer.cc:37-202.
* Config 4's per-GPU share on a graph several times the 2.4 M-state one
  (``bigram_8m``, ~7.7 M states, standing in for vosk-model-en-us-0.22's
  HCLG, src/batch_model.cc:51-54): 256 streams decoded together through the
  pipelined engine with lattices and pruning; every best path equals the C
  oracle's, max-active engaged.
"""
import json
import multiprocessing as mp
import os

import numpy as np
import pytest

import oracle_py
from conftest import perturbed_stream

pytestmark = pytest.mark.gpu

NSTREAMS = 256
_ORC = {}


def _pool_map(fn, n):
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(workers) as pool:
        return pool.map(fn, range(n), chunksize=1)


# ---------------------------------------------------------------- config 3
def _secs(i):
    return 21.0 + 0.5 * (i // 8) % 4 if i % 8 == 0 else 10.0 + 0.01 * i


def _batch_expected_job(i):
    import oracle_endpoint as OE
    import oracle_lattice as OL
    o, info = _ORC["o"], _ORC["info"]
    w = _ORC["waves"][i]
    llh = o.loglikes(w)
    kaldi = oracle_py.decoder_order(batch=True) == "kaldi"
    out = []
    states = []  # the stream's lazy numbering at each segment's start
    segs = OE.batch_segments_fast(o, w, llh, info["right_context"], info["priming"], kaldi=kaldi, lazy_states=states)
    for (s0, s1), ls in zip(segs, states):
        mb = OL.results(o, llh[s0:s1], kaldi=kaldi, lazy_state=ls)["mbr"]
        out.append(dict(text=" ".join(o.words[x] for x in mb["words"]), start=s0 * 0.03,
                        times=[(np.floor(a + 0.5) * 0.03, np.floor(b + 0.5) * 0.03) for a, b in mb["times"]]))
    return out


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


def test_config3_256_batch_recognizers_match_oracle(synth_la_small_en_us, test_wave, tmp_path, monkeypatch):
    import oracle_graph as OG
    import vosk
    from vosk import engine
    vosk.SetLogLevel(-1)
    waves = [perturbed_stream(test_wave, 3000 + i, seconds=_secs(i)) for i in range(NSTREAMS)]
    # ---- the product: the batch API, as test_gpu_batch.py drives it
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_la_small_en_us)
    model = vosk.BatchModel()
    recs = [vosk.BatchRecognizer(model, 16000) for _ in range(NSTREAMS)]
    datas = [_pcm(w) for w in waves]
    got = [[] for _ in range(NSTREAMS)]
    done = [False] * NSTREAMS

    def collect():
        for i in range(NSTREAMS):
            while True:
                r = recs[i].Result()
                if not r:
                    break
                got[i].append(json.loads(r))

    pos = 0
    while not all(done):
        for i in range(NSTREAMS):
            if done[i]:
                continue
            if pos >= len(datas[i]):
                recs[i].FinishStream()
                done[i] = True
            else:
                recs[i].AcceptWaveform(datas[i][pos:pos + 8000])
        pos += 8000
        model.Wait()
        collect()
    model.Wait()
    collect()
    del recs
    # ---- the oracle, on libvosk's static expansion of the same graph pair
    odir, _ = OG.expanded_hclg_model(synth_la_small_en_us, str(tmp_path / "la_hclg"))
    _ORC.update(o=oracle_py.OracleModel(odir, fpc=51), info=engine.plan_info(synth_la_small_en_us, 51),
                waves=waves)
    try:
        exp = _pool_map(_batch_expected_job, NSTREAMS)
    finally:
        _ORC.clear()
    nseg = 0
    for i in range(NSTREAMS):
        g, e = got[i], exp[i]
        assert len(g) == len(e), (i, [r["text"] for r in g], [x["text"] for x in e])
        for r, x in zip(g, e):
            assert r["text"] == x["text"], i
            ws = r.get("result", [])
            assert len(ws) == len(x["times"]), i
            for w, (tb, te) in zip(ws, x["times"]):
                assert w["start"] == pytest.approx(x["start"] + tb, abs=1e-4), i
                assert w["end"] == pytest.approx(x["start"] + te, abs=1e-4), i
        nseg += len(e)
    assert nseg > NSTREAMS  # endpoint segments too
    assert sum(1 for e in exp for x in e if x["text"]) >= NSTREAMS


# ------------------------------------------------- SURVEY §8d's stream shape
def test_section8d_32_streams_of_60s_match_oracle(synth_la_small_en_us, test_wave, tmp_path, monkeypatch):
    """§8d's workload shape: 60-s streams (stream i = test.wav tiled, shifted
    by i * 7919, gain and N(0, 10 LSB) noise from default_rng(1234 + i)), 32
    of them through vosk_batch_* on the bench model, fed the test_gpu_batch.py
    way (8000-byte calls, Wait() and Result() per round, FinishStream at the
    end).  Every result message -- the endpoint segments of the default rules
    (20-s segments), each segment's MBR words and times after Kaldi's pruned
    phone + word determinization -- equals the oracle chain's."""
    import oracle_graph as OG
    import vosk
    from vosk import engine
    vosk.SetLogLevel(-1)
    n = 32
    waves = [perturbed_stream(test_wave, i, seconds=60.0) for i in range(n)]
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_la_small_en_us)
    model = vosk.BatchModel()
    recs = [vosk.BatchRecognizer(model, 16000) for _ in range(n)]
    datas = [_pcm(w) for w in waves]
    got = [[] for _ in range(n)]

    def collect():
        for i in range(n):
            while True:
                r = recs[i].Result()
                if not r:
                    break
                got[i].append(json.loads(r))

    for pos in range(0, len(datas[0]), 8000):
        for i in range(n):
            recs[i].AcceptWaveform(datas[i][pos:pos + 8000])
        model.Wait()
        collect()
    for r in recs:
        r.FinishStream()
    model.Wait()
    collect()
    del recs
    odir, _ = OG.expanded_hclg_model(synth_la_small_en_us, str(tmp_path / "la_hclg"))
    _ORC.update(o=oracle_py.OracleModel(odir, fpc=51), info=engine.plan_info(synth_la_small_en_us, 51),
                waves=waves)
    try:
        exp = _pool_map(_batch_expected_job, n)
    finally:
        _ORC.clear()
    for i in range(n):
        g, e = got[i], exp[i]
        assert len(g) == len(e), (i, [r["text"] for r in g], [x["text"] for x in e])
        for r, x in zip(g, e):
            assert r["text"] == x["text"], i
            ws = r.get("result", [])
            assert len(ws) == len(x["times"]), i
            for w, (tb, te) in zip(ws, x["times"]):
                assert w["start"] == pytest.approx(x["start"] + tb, abs=1e-4), i
                assert w["end"] == pytest.approx(x["start"] + te, abs=1e-4), i
    # the default rules end segments inside every 60-s stream
    assert all(len(e) >= 2 for e in exp)
    assert sum(len(w["text"].split()) for e in exp for w in e) >= 20 * n


# ---------------------------------------------------------------- config 4
def _best_path_job(i):
    r = _ORC["o"].recognize(_ORC["waves"][i])
    return r["path"], int(r["ntok"].max())


def test_config4_256_streams_on_a_7m_state_hclg(synth_bigram_8m, test_wave):
    from vosk import engine
    waves = [perturbed_stream(test_wave, 5000 + i, seconds=4.0 + 0.01 * i) for i in range(NSTREAMS)]
    e = engine.Engine(synth_bigram_8m, frames_per_chunk=51, max_streams=NSTREAMS, pipeline=True, lattice=True)
    e.set_step_samples(51 * 160)
    ss = [e.new_stream() for _ in range(NSTREAMS)]
    for s, w in zip(ss, waves):
        e.preload(s, w, finished=True)
    steps = 0
    while e.step(ss):
        steps += 1
        assert steps < 2000
    paths = []
    for s in ss:
        st = e.decoder_state(s)
        assert st["err"] == 0 and st["lat_ovf"] == 0, st
        paths.append(e.best_path(s, use_final=True)[0])
    e.close()
    o = oracle_py.OracleModel(synth_bigram_8m, fpc=51)
    assert o.graph.num_states > 6_000_000
    _ORC.update(o=o, waves=waves)
    try:
        ref = _pool_map(_best_path_job, NSTREAMS)
    finally:
        _ORC.clear()
    for k in range(NSTREAMS):
        np.testing.assert_array_equal(paths[k], ref[k][0], err_msg=f"stream {k}")
    assert max(r[1] for r in ref) > o.max_active  # max-active engaged
