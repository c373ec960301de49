"""BatchRecognizer endpointing against the oracle (reset_on_endpoint,
src/batch_model.cc:72; PushLattice, src/batch_recognizer.cc:43-107).

Streams of a model whose endpoint rules fire every few seconds are fed the
test_gpu_batch.py way.  Every result message equals the oracle's MBR over
the same decoder segment (tests/oracle_endpoint.batch_segments: the chunk
schedule and the rules after every chunk), with the segment's time offset.
Two feeding patterns: Wait() after every round (the lane runs each batch's
stages in order), and every chunk queued up front (the lane pipelines front
end / nnet / decoder over three HIP streams and applies resets to jobs
already staged): the segment boundaries must not depend on it."""
import json

import numpy as np
import pytest

import batch_expect
from conftest import perturbed_stream

pytestmark = pytest.mark.gpu
N = 6


@pytest.fixture(scope="module")
def vosk_mod():
    import vosk
    vosk.SetLogLevel(-1)
    return vosk


@pytest.fixture(scope="module")
def expected(synth_model_ep, test_wave):
    waves = [perturbed_stream(test_wave, 900 + i, seconds=9.0 + 0.7 * i) for i in range(N)]
    out = batch_expect.expected(synth_model_ep, waves)
    assert sum(len(r) for r in out) >= 3 * N  # the rules fire
    return waves, out


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


@pytest.mark.parametrize("feeding", ["wait_per_round", "queued_upfront"])
def test_batch_endpoint_segments_match_oracle(vosk_mod, synth_model_ep, expected, monkeypatch, feeding):
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_model_ep)
    waves, exp = expected
    model = vosk_mod.BatchModel()
    recs = [vosk_mod.BatchRecognizer(model, 16000) for _ in range(N)]
    datas = [_pcm(w) for w in waves]
    results = [[] for _ in range(N)]

    def collect():
        for i in range(N):
            while True:
                res = recs[i].Result()
                if not res:
                    break
                results[i].append(json.loads(res))

    rounds = max(len(d) for d in datas) // 8000 + 1
    for k in range(rounds):
        for i in range(N):
            chunk = datas[i][k * 8000:(k + 1) * 8000]
            if chunk:
                recs[i].AcceptWaveform(chunk)
        if feeding == "wait_per_round":
            model.Wait()
            collect()
    for r in recs:
        r.FinishStream()
    model.Wait()
    collect()
    for i in range(N):
        assert recs[i].GetPendingChunks() == 0
        batch_expect.check(results[i], exp[i], f"stream {i}")
