"""KaldiRecognizer endpointing against the oracle (src/recognizer.cc:297-323
AcceptWaveform + EndpointDetected :318, Result :808-816, CleanUp :188-224):
a stream fed 8000-byte chunks (test_simple.py) on a model whose endpoint
rules fire every few seconds.  Every Result() taken when AcceptWaveform
returns 1, and the FinalResult, equals the oracle's MBR over the same
decoder segment (oracle_py.OracleModel.online(endpoints=True): the rules
after every call, decoder and silence weighting restarted at the next call,
features and i-vector statistics continuing), with the segment's times (the segment's lattice: the incremental
determinizer's, tests/oracle_incremental.py)."""
import json

import numpy as np
import pytest

from conftest import perturbed_stream
import oracle_incremental as OI
import oracle_py

pytestmark = pytest.mark.gpu


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


@pytest.mark.parametrize("seed", [900, 903])
def test_recognizer_endpoint_segments_match_oracle(synth_model_ep, test_wave, seed):
    import vosk
    vosk.SetLogLevel(-1)
    wave = perturbed_stream(test_wave, seed, seconds=12.0)
    o = oracle_py.OracleModel(synth_model_ep)
    on = o.online(wave, chunk=4000, endpoints=True)
    segs = on["segments"]
    assert len(segs) >= 3  # the rules fire
    # each segment's Result: the incremental determinizer's lattice over the
    # segment (FinalizeDecoding + GetLattice, tests/oracle_incremental.py)
    exp = [(" ".join(o.words[w] for w in ids), [(a, b) for _, a, b, _ in ws])
           for kind, ws, ids in OI.recognizer_run(o, wave, chunk=4000, on=on) if kind == "result"]
    assert len(exp) == len(segs)
    m = vosk.Model(synth_model_ep)
    rec = vosk.KaldiRecognizer(m, 16000)
    rec.SetWords(True)
    data = _pcm(wave)
    got = []
    for i in range(0, len(data), 8000):
        if rec.AcceptWaveform(data[i:i + 8000]):
            got.append(json.loads(rec.Result()))
    got.append(json.loads(rec.FinalResult()))
    assert [g["text"] for g in got] == [e[0] for e in exp]
    for g, (_, times) in zip(got, exp):
        for w, (tb, te) in zip(g.get("result", []), times):
            assert w["start"] == pytest.approx(tb, abs=1e-4)
            assert w["end"] == pytest.approx(te, abs=1e-4)
