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

from conftest import perturbed_stream
import oracle_endpoint as OE
import oracle_lattice as OL
import oracle_py

pytestmark = pytest.mark.gpu
N = 6


@pytest.fixture(scope="module")
def vosk_mod():
    import vosk
    vosk.SetLogLevel(-1)
    return vosk


@pytest.fixture(scope="module")
def expected(synth_model_ep, test_wave):
    from vosk import engine
    info = engine.plan_info(synth_model_ep, 51)
    o = oracle_py.OracleModel(synth_model_ep, fpc=51)
    waves = [perturbed_stream(test_wave, 900 + i, seconds=9.0 + 0.7 * i) for i in range(N)]
    out = []
    for w in waves:
        llh = o.loglikes(w)
        kaldi = oracle_py.decoder_order(batch=True) == "kaldi"
        segs = OE.batch_segments_fast(o, w, llh, info["right_context"], info["priming"], kaldi=kaldi)
        res = []
        for s0, s1 in segs:
            mb = OL.results(o, llh[s0:s1], kaldi=kaldi)["mbr"]
            res.append(dict(text=" ".join(o.words[x] for x in mb["words"]), start=s0 * 0.03,
                            times=[(np.floor(a + 0.5) * 0.03, np.floor(b + 0.5) * 0.03) for a, b in mb["times"]]))
        out.append(res)
    assert sum(len(r) for r in out) >= 3 * N  # the rules fire
    return waves, out


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


def _check(results, exp):
    assert len(results) == len(exp), ([r["text"] for r in results], [e["text"] for e in exp])
    for r, e in zip(results, exp):
        assert r["text"] == e["text"]
        for w, (tb, te) in zip(r.get("result", []), e["times"]):
            assert w["start"] == pytest.approx(e["start"] + tb, abs=1e-4)
            assert w["end"] == pytest.approx(e["start"] + te, abs=1e-4)


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
        _check(results[i], exp[i])
