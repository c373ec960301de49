"""Every output of the reference's test_simple.py loop (python/example:
AcceptWaveform on 8000-byte chunks, Result() when it returns 1, else
PartialResult(), then FinalResult()) through libvosk.so's KaldiRecognizer,
against the oracle chain (tests/oracle_incremental.recognizer_run): the
decoder segments, each partial result -- the best path's words without
partial words (GetBestPath(false) + GetLinearSymbolSequence,
src/recognizer.cc:782-800), the incremental determinizer's lattice with them
("" until NumFramesInLattice() > 0, then GetLattice(NumFramesInLattice(),
false), WordAlignLatticePartial and MBR, :740-780) -- and every result
(FinalizeDecoding + GetLattice(NumFramesDecoded(), true) over the
incremental determinizer, graph scale 0.9, word alignment, MBR, :669-729):
texts, word times and confidences."""
import json

import numpy as np
import pytest

from conftest import perturbed_stream
import oracle_incremental as OI
import oracle_py

pytestmark = pytest.mark.gpu


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


def _run_library(model, wave, partial_words):
    import vosk
    vosk.SetLogLevel(-1)
    m = vosk.Model(model)
    rec = vosk.KaldiRecognizer(m, 16000)
    rec.SetWords(True)
    rec.SetPartialWords(partial_words)
    data = _pcm(wave)
    got = []
    for i in range(0, len(data), 8000):
        if rec.AcceptWaveform(data[i:i + 8000]):
            got.append(("result", json.loads(rec.Result())))
        else:
            got.append(("partial", json.loads(rec.PartialResult())))
    got.append(("result", json.loads(rec.FinalResult())))
    return got


def _compare(o, got, exp, partial_words):
    assert [k for k, _ in got] == [e[0] for e in exp]
    nwords = 0
    for i, ((kind, g), (_, ws, ids)) in enumerate(zip(got, exp)):
        text = " ".join(o.words[w] for w in ids)
        if kind == "partial":
            assert g["partial"] == text, i
            if not partial_words:
                assert "partial_result" not in g
                continue
            gw = g.get("partial_result", [])
        else:
            assert g["text"] == text, i
            gw = g.get("result", [])
        assert [w["word"] for w in gw] == [o.words[w[0]] for w in ws], i
        for w, (_, st, en, cf) in zip(gw, ws):
            assert w["start"] == pytest.approx(st, abs=1e-4), i
            assert w["end"] == pytest.approx(en, abs=1e-4), i
            assert w["conf"] == pytest.approx(float(cf), abs=2e-6), i
        nwords += len(gw)
    return nwords


@pytest.mark.parametrize("partial_words", [False, True])
def test_test_simple_outputs_long_segment(synth_model, test_wave, partial_words):
    """One 15-s decoder segment (no endpoint fires on the base model): many
    incremental chunks, partial results from the determinized chunks."""
    wave = perturbed_stream(test_wave, 31, seconds=15.0)
    o = oracle_py.OracleModel(synth_model)
    exp = OI.recognizer_run(o, wave, chunk=4000, partial_words=partial_words)
    got = _run_library(synth_model, wave, partial_words)
    assert _compare(o, got, exp, partial_words) > 10
    partials = [g["partial"] for k, g in got if k == "partial"]
    assert any(partials)
    if partial_words:  # "" until the first chunk is determinized (>= 60 frames = 1.8 s)
        assert partials[:6] == [""] * 6


def test_test_simple_outputs_compacted_records(synth_model, test_wave, monkeypatch):
    """Arenas a fraction of the segment's records (64 K tokens, 128 K links
    per stream; the 15-s segment makes ~230 K tokens, ~280 K links): the
    engine's pruning pass compacts them many times while the incremental
    lattice reads them (gated on the frames the host has read,
    Engine::SetHostRead) -- every output still equals the oracle chain's, no
    best-path fallback."""
    monkeypatch.setenv("VOSK_AMD_REC_ARENA_TOKENS", str(1 << 16))
    monkeypatch.setenv("VOSK_AMD_REC_LINKS", str(1 << 17))
    wave = perturbed_stream(test_wave, 31, seconds=15.0)
    o = oracle_py.OracleModel(synth_model)
    exp = OI.recognizer_run(o, wave, chunk=4000, partial_words=True)
    got = _run_library(synth_model, wave, True)
    assert _compare(o, got, exp, True) > 10


@pytest.mark.parametrize("partial_words", [False, True])
def test_test_simple_outputs_with_endpoints(synth_model_ep, test_wave, partial_words):
    """Endpoints every few seconds: each Result() closes a decoder segment,
    the next call starts a new incremental lattice (CleanUp)."""
    wave = perturbed_stream(test_wave, 900, seconds=12.0)
    o = oracle_py.OracleModel(synth_model_ep)
    exp = OI.recognizer_run(o, wave, chunk=4000, partial_words=partial_words)
    got = _run_library(synth_model_ep, wave, partial_words)
    assert sum(1 for k, _ in got if k == "result") >= 4
    assert _compare(o, got, exp, partial_words) > 5
