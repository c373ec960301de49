"""GPU final lattice prune of ending batch segments (decoder.hip
prune_final_kernel; Kaldi FinalizeDecoding / PruneForwardLinksFinal): the
segments' records shrink before their copy, and every result message is the
same as without it (the host's exact lattice-beam prune keeps exactly what it
kept).  Reference: src/batch_recognizer.cc:43-107 (results from the
segment's lattice)."""
import json

import numpy as np
import pytest

from conftest import perturbed_stream

pytestmark = pytest.mark.gpu


def _run(vosk, model_dir, waves, monkeypatch, final_prune):
    from vosk import engine
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", model_dir)
    monkeypatch.setenv("VOSK_AMD_FINAL_PRUNE", "1" if final_prune else "0")
    model = vosk.BatchModel()
    recs = [vosk.BatchRecognizer(model, 16000) for _ in waves]
    datas = [np.asarray(w, np.float32).astype("<i2").tobytes() for w in waves]
    out = [[] for _ in waves]
    done = [False] * len(waves)

    def collect():
        for i, r in enumerate(recs):
            while True:
                x = r.Result()
                if not x:
                    break
                out[i].append(json.loads(x))

    pos = 0
    while not all(done):
        for i, d in enumerate(datas):
            if done[i]:
                continue
            if pos >= len(d):
                recs[i].FinishStream()
                done[i] = True
            else:
                recs[i].AcceptWaveform(d[pos:pos + 8000])
        pos += 8000
        model.Wait()
        collect()
    model.Wait()
    collect()
    prof = engine.batch_result_profile(model)
    del recs
    return out, prof


def test_final_prune_keeps_results_and_shrinks_copies(synth_model_ep, test_wave, monkeypatch):
    import vosk
    vosk.SetLogLevel(-1)
    waves = [perturbed_stream(test_wave, 700 + i, seconds=6.0 + 1.5 * i) for i in range(12)]
    plain, p0 = _run(vosk, synth_model_ep, waves, monkeypatch, False)
    pruned, p1 = _run(vosk, synth_model_ep, waves, monkeypatch, True)
    assert p0["segments"] == p1["segments"] > len(waves)  # endpoint segments too
    assert p1["links_copied"] < p0["links_copied"]
    for a, b in zip(plain, pruned):
        assert [x["text"] for x in a] == [x["text"] for x in b]
        for x, y in zip(a, b):
            wx, wy = x.get("result", []), y.get("result", [])
            assert [w["word"] for w in wx] == [w["word"] for w in wy]
            for u, v in zip(wx, wy):
                assert u["conf"] == pytest.approx(v["conf"], abs=1e-6)
                assert u["start"] == v["start"] and u["end"] == v["end"]
