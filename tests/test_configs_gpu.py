"""BASELINE configs 4 and 5 at their per-GPU shape through the public API
(VERDICT r03 item 3).

* Config 4 (2048 streams / 8 GPUs, vosk-model-en-us-0.22): 256
  ``BatchRecognizer``s on one GPU through ``vosk_batch_*`` over a graph of
  several million states (``bigram_8m``, ~7.7 M states, standing in for
  en-us-0.22's HCLG, src/batch_model.cc:51-54).  Every result message --
  segment boundaries, MBR words and word times -- equals the oracle's: the
  batch segmentation restated per chunk (oracle_endpoint), then each
  segment's lattice through the Python result chain (oracle_lattice).
* Config 5 (1024 streams / 8 GPUs, ru + speaker model): 128 KaldiRecognizers
  with a speaker model on 128 threads (src/recognizer.cc:326-419,470-479);
  every final result's text, "spk" vector and "spk_frames" equal the
  oracle's (the online decode's best path selects the frames,
  tests/oracle_xvector.py extracts the x-vector).
"""
import json
import multiprocessing as mp
import os
import threading

import numpy as np
import pytest

import oracle_py
from conftest import perturbed_stream

pytestmark = pytest.mark.gpu

_ORC = {}


def _pool_map(fn, n):
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("fork").Pool(workers) as pool:
        return pool.map(fn, range(n), chunksize=1)


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


def run_batch_api(model_dir, waves, monkeypatch, feed=8000):
    """The reference's test_gpu_batch.py loop over `waves`: every result
    message of every stream (FinishStream at each stream's end)."""
    import vosk
    vosk.SetLogLevel(-1)
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", model_dir)
    model = vosk.BatchModel()
    recs = [vosk.BatchRecognizer(model, 16000) for _ in waves]
    datas = [_pcm(w) for w in waves]
    got = [[] for _ in waves]
    done = [False] * len(waves)

    def collect():
        for i, r in enumerate(recs):
            while True:
                x = r.Result()
                if not x:
                    break
                got[i].append(json.loads(x))

    pos = 0
    while not all(done):
        for i in range(len(waves)):
            if done[i]:
                continue
            if pos >= len(datas[i]):
                recs[i].FinishStream()
                done[i] = True
            else:
                recs[i].AcceptWaveform(datas[i][pos:pos + feed])
        pos += feed
        model.Wait()
        collect()
    model.Wait()
    collect()
    del recs
    del model
    return got


def _batch_expected_job(i):
    import oracle_endpoint as OE
    import oracle_lattice as OL
    o, info = _ORC["o"], _ORC["info"]
    w = _ORC["waves"][i]
    llh = o.loglikes(w)
    kaldi = oracle_py.decoder_order(batch=True) == "kaldi"
    out = []
    for s0, s1 in OE.batch_segments_fast(o, w, llh, info["right_context"], info["priming"], kaldi=kaldi):
        mb = OL.results(o, llh[s0:s1], kaldi=kaldi)["mbr"]
        out.append(dict(text=" ".join(o.words[x] for x in mb["words"]), start=s0 * 0.03,
                        times=[(np.floor(a + 0.5) * 0.03, np.floor(b + 0.5) * 0.03) for a, b in mb["times"]]))
    return out


def compare_batch_results(got, exp):
    nseg = 0
    for i in range(len(got)):
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
    return nseg


def test_config4_256_batch_recognizers_on_a_7m_state_hclg(synth_bigram_8m, test_wave, monkeypatch):
    from vosk import engine
    n = 256
    waves = [perturbed_stream(test_wave, 7000 + i, seconds=4.0 + 0.02 * i) for i in range(n)]
    got = run_batch_api(synth_bigram_8m, waves, monkeypatch)
    o = oracle_py.OracleModel(synth_bigram_8m, fpc=51)
    assert o.graph.num_states > 6_000_000
    _ORC.update(o=o, info=engine.plan_info(synth_bigram_8m, 51), waves=waves)
    try:
        exp = _pool_map(_batch_expected_job, n)
    finally:
        _ORC.clear()
    assert compare_batch_results(got, exp) >= n
    assert sum(1 for e in exp for x in e if x["text"]) >= n // 2


# ---------------------------------------------------------------- config 5
def _spk_expected_job(i):
    import oracle_incremental as OI
    o, ox, sil = _ORC["o"], _ORC["ox"], _ORC["sil"]
    w = _ORC["waves"][i]
    on = o.online(w, chunk=4000)
    dec = on["decode"]
    g, tm = o.graph, o.tm
    keep = [0 if int(tm.tid2phone[g.ilabel[a]]) in sil else 1 for a in dec["path"] if g.ilabel[a] != 0]
    ref, nr = ox.xvector(w, 0, keep)
    # the final result's text: MBR over the incremental determinizer's lattice
    mb = OI.final_result(o, w, 4000, on=on)["mbr"]
    return " ".join(o.words[x] for x in mb["words"]), (None if ref is None else ref.astype(np.float64)), nr


def test_config5_128_speaker_recognizers_match_oracle(synth_model_noep, synth_spk, test_wave):
    import oracle_xvector as OX
    import vosk
    vosk.SetLogLevel(-1)
    n = 128
    waves = [perturbed_stream(test_wave, 9000 + i, seconds=5.0 + 0.02 * i) for i in range(n)]
    m = vosk.Model(synth_model_noep)
    spk = vosk.SpkModel(synth_spk)
    recs = [vosk.KaldiRecognizer(m, 16000, spk) for _ in range(n)]
    out, errs = {}, []

    def work(i):
        try:
            d = _pcm(waves[i])
            for k in range(0, len(d), 8000):
                recs[i].AcceptWaveform(d[k:k + 8000])
            out[i] = json.loads(recs[i].FinalResult())
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in th) and not errs, errs
    del recs
    o = oracle_py.OracleModel(synth_model_noep)
    sil = set(int(p) for p in str(o.model_conf.get("endpoint.silence-phones", "")).replace(",", ":").split(":") if p)
    _ORC.update(o=o, ox=OX.OracleSpk(synth_spk), sil=sil, waves=waves)
    try:
        exp = _pool_map(_spk_expected_job, n)
    finally:
        _ORC.clear()
    n_spk = 0
    for i in range(n):
        text, ref, nr = exp[i]
        r = out[i]
        assert r["text"] == text, i
        if ref is None:
            assert "spk" not in r, i
            continue
        n_spk += 1
        assert r["spk_frames"] == nr, i
        np.testing.assert_allclose(np.array(r["spk"], np.float64), ref, atol=1e-6, err_msg=f"stream {i}")
    assert n_spk >= n // 2
