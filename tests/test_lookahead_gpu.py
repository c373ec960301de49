"""Lookahead models and grammar recognizers on the GPU.

The engine loads a lookahead model directory (graph/HCLr.fst + graph/Gr.fst,
no HCLG) and decodes on the static expansion of HCLr o Gr; the C oracle
decodes a copy of the model whose graph/HCLG.fst is the unpruned
restatement of that composition (tests/oracle_graph.py), so the comparison
is the usual bit-exact one (tokens, costs, best path, lattice-based
results).  The grammar recognizer (vosk_recognizer_new_grm) is checked the
same way against HCLr o (phrase-list bigram).
"""
import json

import numpy as np
import pytest

from conftest import perturbed_stream
import oracle_graph as OG
import oracle_py

pytestmark = pytest.mark.gpu

GRAMMAR = '["w00001 w00002 w00003", "w00004 w00005", "w00006", "w00007 w00001", "w00008 w00009 w00010"]'


@pytest.fixture(scope="module")
def vosk_mod():
    import vosk
    vosk.SetLogLevel(-1)
    return vosk


@pytest.fixture(scope="module")
def la_oracle(synth_lookahead, tmp_path_factory):
    d = OG.write_hclg_model(synth_lookahead, str(tmp_path_factory.mktemp("la") / "hclg"))
    return oracle_py.OracleModel(d)


@pytest.fixture(scope="module")
def grammar_oracle(synth_lookahead, tmp_path_factory):
    d = OG.write_hclg_model(synth_lookahead, str(tmp_path_factory.mktemp("lag") / "hclg"), GRAMMAR)
    return oracle_py.OracleModel(d)


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


def test_lookahead_engine_matches_oracle(synth_lookahead, la_oracle, test_wave):
    from vosk import engine
    e = engine.Engine(synth_lookahead, frames_per_chunk=0, max_streams=4, stats=True, keep_llh=True)
    waves = [test_wave, perturbed_stream(test_wave, 3, seconds=6.0)]
    for w in waves:
        s = e.new_stream()
        for i in range(0, len(w), 3200):
            e.accept(s, w[i:i + 3200])
            e.advance([s])
        e.accept(s, np.zeros(0, np.float32), finished=True)
        e.advance([s])
        r = la_oracle.recognize(w)
        arcs, cost, _ = e.best_path(s, use_final=True)
        np.testing.assert_array_equal(arcs, r["path"])
        assert e.frames_decoded(s) == len(r["ntok"]) - 1
        assert e.error(s) == 0


def _final_text(vosk_mod, model, wave, grammar=None):
    rec = vosk_mod.KaldiRecognizer(model, 16000, grammar) if grammar else vosk_mod.KaldiRecognizer(model, 16000)
    rec.SetWords(True)
    data = _pcm(wave)
    for i in range(0, len(data), 8000):
        assert rec.AcceptWaveform(data[i:i + 8000]) == 0  # endpointing disabled
    return json.loads(rec.FinalResult())


def _oracle_text(oracle, wave):
    import oracle_incremental as OI  # the recognizer's incremental lattice
    mb = OI.final_result(oracle, wave, 4000)["mbr"]
    return " ".join(oracle.words[w] for w in mb["words"])


def test_lookahead_recognizer_matches_oracle(vosk_mod, synth_lookahead, la_oracle, test_wave):
    m = vosk_mod.Model(synth_lookahead)
    final = _final_text(vosk_mod, m, test_wave)
    assert final["text"] == _oracle_text(la_oracle, test_wave)
    assert final["text"]


def test_grammar_recognizer_matches_oracle(vosk_mod, synth_lookahead, grammar_oracle, test_wave):
    m = vosk_mod.Model(synth_lookahead)
    allowed = set(" ".join(json.loads(GRAMMAR)).split())
    for k, w in enumerate([test_wave, perturbed_stream(test_wave, 5, seconds=5.0)]):
        final = _final_text(vosk_mod, m, w, GRAMMAR)
        assert final["text"] == _oracle_text(grammar_oracle, w), k
        assert set(final["text"].split()) <= allowed
    # recognizers with the same grammar share its engine; a plain recognizer
    # on the same model keeps the full graph
    r1 = vosk_mod.KaldiRecognizer(m, 16000, GRAMMAR)
    r2 = vosk_mod.KaldiRecognizer(m, 16000, GRAMMAR)
    del r1, r2
    full = _final_text(vosk_mod, m, test_wave)
    assert not set(full["text"].split()) <= allowed or full["text"] == ""


def test_bad_grammar_fails_to_create(vosk_mod, synth_lookahead):
    m = vosk_mod.Model(synth_lookahead)
    with pytest.raises(Exception):
        vosk_mod.KaldiRecognizer(m, 16000, "[1, 2]")


def test_grammar_on_hclg_model_uses_static_graph(vosk_mod, synth_model_noep, test_wave):
    """src/recognizer.cc:96-98: a model without HCLr warns and decodes with
    its HCLG."""
    m = vosk_mod.Model(synth_model_noep)
    a = _final_text(vosk_mod, m, test_wave[:48000], '["w00001"]')
    b = _final_text(vosk_mod, m, test_wave[:48000])
    assert a == b


def test_batch_recognizer_on_a_lookahead_model(vosk_mod, synth_lookahead, la_oracle, test_wave, monkeypatch):
    """BASELINE config 3 names vosk-model-small-en-us, which ships HCLr.fst +
    Gr.fst: the reference's CUDA batch path needs an HCLG; here the
    BatchModel decodes on the expanded graph.  Final texts == the oracle's
    MBR words on that graph (test_gpu_batch.py pattern)."""
    import oracle_lattice as OL
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_lookahead)
    oracle = oracle_py.OracleModel(la_oracle.dir, fpc=51)
    vosk_mod.GpuInit()
    model = vosk_mod.BatchModel()
    n = 4
    waves = [perturbed_stream(test_wave, i, seconds=2.5 + 0.5 * i) for i in range(n)]
    recs = [vosk_mod.BatchRecognizer(model, 16000) for _ in range(n)]
    datas = [_pcm(w) for w in waves]
    pos, texts, ended = [0] * n, [""] * n, set()
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
        mb = OL.results(oracle, oracle.loglikes(waves[i]), kaldi=oracle_py.decoder_order(batch=True) == "kaldi")["mbr"]
        assert texts[i] == " ".join(oracle.words[w] for w in mb["words"]), i
