"""Public API on the GPU: the reference harness patterns (test_simple.py,
test_gpu_batch.py, c/test_vosk.c) through the Python binding and the C ABI,
checked against the CPU oracle's 1-best transcript."""
import ctypes as C
import json
import os

import numpy as np
import pytest

from conftest import perturbed_stream
import oracle_py

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vosk_mod():
    import vosk
    vosk.SetLogLevel(-1)
    return vosk


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


def _oracle_mbr(oracle, wave, chunk):
    # the recognizer's final result: the incremental determinizer's lattice
    # (src/recognizer.cc:678; tests/oracle_incremental.py)
    import oracle_incremental as OI
    return OI.final_result(oracle, wave, chunk)["mbr"]


def _oracle_mbr_text(oracle, wave, batch=False):
    import oracle_lattice as OL
    mb = OL.results(oracle, oracle.loglikes(wave), kaldi=oracle_py.decoder_order(batch) == "kaldi")["mbr"]
    return " ".join(oracle.words[w] for w in mb["words"])


def test_kaldi_recognizer_matches_oracle(vosk_mod, synth_model_noep, test_wave):
    """test_simple.py pattern: 4000-frame chunks, partial results, final result.
    The reference Recognizer silence-weights its i-vector statistics from the
    decoder's best path (src/recognizer.cc:226-237): the oracle replays the
    same online flow."""
    oracle = oracle_py.OracleModel(synth_model_noep)
    ref = oracle.online(test_wave, chunk=4000)["decode"]
    ref["text"] = " ".join(oracle.words[w] for w in ref["words"])
    m = vosk_mod.Model(synth_model_noep)
    rec = vosk_mod.KaldiRecognizer(m, 16000)
    rec.SetWords(True)
    rec.SetPartialWords(True)
    data = _pcm(test_wave)
    partials = []
    for i in range(0, len(data), 8000):
        assert rec.AcceptWaveform(data[i:i + 8000]) == 0  # endpointing disabled
        p = json.loads(rec.PartialResult())
        assert "partial" in p
        partials.append(p["partial"])
    final = json.loads(rec.FinalResult())
    # the result is the MBR decoding of the segment's lattice (graph scale
    # 0.9, src/recognizer.cc:429-482,718): words, confidences, times
    mb = _oracle_mbr(oracle, test_wave, 4000)
    assert final["text"] == " ".join(oracle.words[w] for w in mb["words"])
    assert [w["word"] for w in final.get("result", [])] == final["text"].split()
    for w, c, (tb, te) in zip(final.get("result", []), mb["conf"], mb["times"]):
        assert w["conf"] == pytest.approx(c, abs=1e-5)
        assert w["start"] == pytest.approx(tb * 0.03, abs=1e-5)
        assert w["end"] == pytest.approx(te * 0.03, abs=1e-5)
        assert 0.0 <= w["start"] <= w["end"] <= len(test_wave) / 16000 + 0.1
    assert any(partials)  # partial hypotheses appear while streaming
    # next AcceptWaveform after FinalResult starts a fresh utterance
    assert rec.AcceptWaveform(data[:16000]) == 0
    assert isinstance(json.loads(rec.PartialResult())["partial"], str)
    final2 = json.loads(rec.FinalResult())
    ref2 = oracle.online(test_wave[:8000], chunk=8000)["decode"]
    assert final2["text"] == " ".join(oracle.words[w] for w in ref2["words"])


def test_accept_waveform_variants_agree(vosk_mod, synth_model_noep, test_wave):
    m = vosk_mod.Model(synth_model_noep)
    lib = vosk_mod._c
    x = test_wave[:48000]
    outs = []
    for kind in ("c", "s", "f"):
        r = lib.vosk_recognizer_new(m._handle, 16000.0)
        assert r
        if kind == "c":
            b = _pcm(x)
            lib.vosk_recognizer_accept_waveform(r, b, len(b))
        elif kind == "s":
            s = np.ascontiguousarray(x.astype(np.int16))
            lib.vosk_recognizer_accept_waveform_s(r, s.ctypes.data, len(s))
        else:
            f = np.ascontiguousarray(x, np.float32)
            lib.vosk_recognizer_accept_waveform_f(r, f.ctypes.data, len(f))
        outs.append(lib.vosk_recognizer_final_result(r).decode())
        lib.vosk_recognizer_free(r)
    assert outs[0] == outs[1] == outs[2]


def test_empty_results_format(vosk_mod, synth_model_noep):
    m = vosk_mod.Model(synth_model_noep)
    rec = vosk_mod.KaldiRecognizer(m, 16000)
    assert rec.Result() == '{"text": ""}'           # src/recognizer.cc:858
    assert rec.FinalResult() == '{"text": ""}'
    rec.SetMaxAlternatives(3)
    assert rec.FinalResult() == '{"alternatives" : [{"text": "", "confidence" : 1.0}] }'
    assert vosk_mod.KaldiRecognizer(m, 16000).PartialResult() == '{"text": ""}'


def test_endpointing_segments(vosk_mod, synth_model, test_wave):
    """With the model's endpoint rules active, results come in segments and
    every segment is a well-formed result."""
    m = vosk_mod.Model(synth_model)
    rec = vosk_mod.KaldiRecognizer(m, 16000)
    data = _pcm(np.concatenate([test_wave, test_wave]))
    results = []
    for i in range(0, len(data), 8000):
        if rec.AcceptWaveform(data[i:i + 8000]):
            results.append(json.loads(rec.Result()))
    results.append(json.loads(rec.FinalResult()))
    assert all("text" in r for r in results)


def test_batch_recognizer_matches_oracle(vosk_mod, synth_model_noep, test_wave, monkeypatch):
    """test_gpu_batch.py pattern: N streams fed 8000 bytes per iteration,
    Wait(), Result(); final text per stream == oracle 1-best."""
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_model_noep)
    # BatchModel chunking: frames_per_chunk = max(51, right context) (batch_model.cc:84-88)
    oracle = oracle_py.OracleModel(synth_model_noep, fpc=51)
    vosk_mod.GpuInit()
    model = vosk_mod.BatchModel()
    n = 6
    waves = [perturbed_stream(test_wave, i, seconds=2.0 + 0.45 * i) for i in range(n)]
    recs = [vosk_mod.BatchRecognizer(model, 16000) for _ in range(n)]
    datas = [_pcm(w) for w in waves]
    pos = [0] * n
    texts = [""] * n
    ended = set()
    while len(ended) < n:
        for i in range(n):
            if i in ended:
                continue
            chunk = datas[i][pos[i]:pos[i] + 8000]
            pos[i] += 8000
            if not chunk:
                recs[i].FinishStream()
                ended.add(i)
                continue
            recs[i].AcceptWaveform(chunk)
        model.Wait()
        for i in range(n):
            res = recs[i].Result()
            if res:
                texts[i] = (texts[i] + " " + json.loads(res)["text"]).strip()
    model.Wait()
    for i in range(n):
        res = recs[i].Result()
        if res:
            texts[i] = (texts[i] + " " + json.loads(res)["text"]).strip()
        assert recs[i].GetPendingChunks() == 0
        # PushLattice: the MBR words of the stream's lattice (batch_recognizer.cc:43-107)
        assert texts[i] == _oracle_mbr_text(oracle, waves[i], batch=True), i


def test_alternatives_and_nlsml_from_lattice(vosk_mod, synth_model_noep, test_wave):
    """SetMaxAlternatives: the n-best word sequences of the segment's lattice
    with likelihood -(graph + acoustic) (NbestResult, src/recognizer.cc:526-
    607); NLSML carries the same texts and likelihoods (:609-667)."""
    import oracle_incremental as OI
    oracle = oracle_py.OracleModel(synth_model_noep)
    x = test_wave[:16000 * 5]
    nb = OI.final_result(oracle, x, 4000, nbest_n=3)["nbest"]
    m = vosk_mod.Model(synth_model_noep)
    outs = {}
    for nlsml in (False, True):
        rec = vosk_mod.KaldiRecognizer(m, 16000)
        rec.SetMaxAlternatives(3)
        rec.SetWords(True)
        rec.SetNLSML(nlsml)
        data = _pcm(x)
        for i in range(0, len(data), 8000):
            rec.AcceptWaveform(data[i:i + 8000])
        outs[nlsml] = rec.FinalResult()
    alts = json.loads(outs[False])["alternatives"]
    assert [a["text"] for a in alts] == [" ".join(oracle.words[w] for w in p["words"]) for p in nb]
    for a, p in zip(alts, nb):
        assert a["confidence"] == pytest.approx(-(p["graph"] + p["acoustic"]), abs=1e-2)
        assert [w["word"] for w in a.get("result", [])] == a["text"].split()
    assert outs[True].startswith('<?xml version="1.0"?>\n<result grammar="default">\n')
    assert outs[True].count("<interpretation") == len(alts)
    for a in alts:
        assert "<instance>" + a["text"] + "</instance>" in outs[True]
