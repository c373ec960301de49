"""BASELINE config 5's shape on one GPU: many KaldiRecognizers with a speaker
model (vosk_recognizer_new_spk), one per thread.  Their decoding shares
batched engine passes (RecognizerGroup) and their x-vectors run on the
model's GPU extractor; every stream's texts, speaker vectors and frame
counts must equal those of the same stream decoded alone."""
import json
import threading

import numpy as np
import pytest

from conftest import perturbed_stream

pytestmark = pytest.mark.gpu

N = 12


def _run(rec, data, out, key):
    res = []
    for i in range(0, len(data), 8000):
        if rec.AcceptWaveform(data[i:i + 8000]):
            res.append(json.loads(rec.Result()))
    res.append(json.loads(rec.FinalResult()))
    out[key] = res


def test_concurrent_speaker_recognizers_match_sequential(synth_model_ep, synth_spk, test_wave):
    import vosk
    vosk.SetLogLevel(-1)
    m = vosk.Model(synth_model_ep)
    spk = vosk.SpkModel(synth_spk)
    waves = [np.asarray(perturbed_stream(test_wave, 500 + i, seconds=8.0), np.float32).astype("<i2").tobytes()
             for i in range(N)]
    alone = {}
    for i, d in enumerate(waves):
        _run(vosk.KaldiRecognizer(m, 16000, spk), d, alone, i)
    recs = [vosk.KaldiRecognizer(m, 16000, spk) for _ in range(N)]
    together, errs = {}, []

    def work(i):
        try:
            _run(recs[i], waves[i], together, i)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(N)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    assert not any(t.is_alive() for t in th) and not errs, errs
    n_spk = 0
    for i in range(N):
        assert len(together[i]) == len(alone[i])
        for a, b in zip(alone[i], together[i]):
            assert a["text"] == b["text"]
            assert a.get("spk_frames") == b.get("spk_frames")
            if "spk" in a:
                n_spk += 1
                np.testing.assert_array_equal(np.array(a["spk"]), np.array(b["spk"]))
    assert n_spk > 0  # speaker vectors were produced
