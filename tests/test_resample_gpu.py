"""Input-rate conversion on the GPU (A3): features of a resampled stream and
an 8 kHz KaldiRecognizer against the oracle (resample -> MFCC -> decode)."""
import json

import numpy as np
import pytest

import oracle_py

pytestmark = pytest.mark.gpu


def _at_rate(wave16k, rate):
    """Test input at another rate (any interpolation will do: it is only data)."""
    n = int(len(wave16k) * rate / 16000)
    t = np.arange(n) * (16000.0 / rate)
    return np.round(np.interp(t, np.arange(len(wave16k)), wave16k)).astype(np.float32)


@pytest.mark.parametrize("rate", [8000, 22050, 44100, 48000])
def test_resampled_features_bit_exact(synth_model, test_wave, rate):
    from vosk import engine
    o = oracle_py.OracleModel(synth_model)
    x = _at_rate(test_wave[:32000], rate)
    ref = o.features(oracle_py.resample(x, rate, 16000))
    e = engine.Engine(synth_model, max_streams=2)
    s = e.new_stream()
    e.set_rate(s, rate)
    step = 1237  # odd chunks: outputs span chunk boundaries
    for i in range(0, len(x), step):
        e.accept(s, x[i:i + step])
        e.advance([s])
    e.accept(s, np.zeros(0, np.float32), finished=True)
    e.advance([s])
    n = ref.shape[0]
    got = e.features(s, 0, n, ref.shape[1])
    np.testing.assert_array_equal(got, ref)


def test_recognizer_8khz_matches_oracle(synth_model_noep, test_wave):
    import vosk
    vosk.SetLogLevel(-1)
    o = oracle_py.OracleModel(synth_model_noep)
    x = _at_rate(test_wave, 8000)
    r = o.online(x, chunk=2000, rate=8000)["decode"]  # silence-weighted online flow
    ref = dict(text=" ".join(o.words[w] for w in r["words"]))
    m = vosk.Model(synth_model_noep)
    rec = vosk.KaldiRecognizer(m, 8000)
    data = x.astype("<i2").tobytes()
    for i in range(0, len(data), 4000):
        rec.AcceptWaveform(data[i:i + 4000])
    assert json.loads(rec.FinalResult())["text"] == ref["text"]


@pytest.mark.parametrize("rate,call_bytes", [(8000, 4000), (44100, 8000), (22050, 3000)])
def test_batch_recognizer_resamples_each_call(synth_model_noep, test_wave, monkeypatch, rate, call_bytes):
    """BatchRecognizer at another rate: each AcceptWaveform call resampled on
    its own with the end flush (LinearResample::Resample(input, true),
    src/batch_recognizer.cc:27-29,157-158), the model-rate samples chunked.
    The oracle: each call through the whole-signal resampler, concatenated,
    decoded (batch order), MBR text of the lattice."""
    import vosk
    import oracle_lattice as OL
    vosk.SetLogLevel(-1)
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_model_noep)
    o = oracle_py.OracleModel(synth_model_noep, fpc=51)
    vosk.GpuInit()
    model = vosk.BatchModel()
    n = 3
    waves = [_at_rate(test_wave[int(16000 * 0.7 * i):], rate)[:int(rate * (3.0 + 0.6 * i))] for i in range(n)]
    datas = [x.astype("<i2").tobytes() for x in waves]
    recs = [vosk.BatchRecognizer(model, rate) for _ in range(n)]
    texts = [""] * n
    pos = [0] * n
    ended = set()
    while len(ended) < n:
        for i in range(n):
            if i in ended:
                continue
            chunk = datas[i][pos[i]:pos[i] + call_bytes]
            pos[i] += call_bytes
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
        x = waves[i]
        step = call_bytes // 2
        y = np.concatenate([oracle_py.resample(x[j:j + step], rate, 16000) for j in range(0, len(x), step)])
        mb = OL.results(o, o.loglikes(y), kaldi=oracle_py.decoder_order(batch=True) == "kaldi")["mbr"]
        assert texts[i] == " ".join(o.words[w] for w in mb["words"]), (i, texts[i])
        assert texts[i]


def test_batch_rate_table_overflow_leaves_the_lane_usable(synth_model_noep, test_wave, monkeypatch):
    """A lane holds kMaxResampleTables (32) input rates: the recognizer at a
    33rd rate fails to construct, and the lane keeps no pointer to it (its
    slot is released before the constructor rethrows); the other recognizers
    keep decoding."""
    import vosk
    vosk.SetLogLevel(-1)
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_model_noep)
    vosk.GpuInit()
    model = vosk.BatchModel()
    recs = [vosk.BatchRecognizer(model, 8000 + 250 * i) for i in range(32)]  # 8000 .. 15750 Hz
    with pytest.raises(Exception):
        vosk.BatchRecognizer(model, 7000)
    rec = vosk.BatchRecognizer(model, 16000)
    data = test_wave[:16000 * 3].astype("<i2").tobytes()
    for i in range(0, len(data), 8000):
        rec.AcceptWaveform(data[i:i + 8000])
        recs[0].AcceptWaveform(data[i // 2:i // 2 + 4000])
        model.Wait()
        rec.Result()
        recs[0].Result()
    rec.FinishStream()
    recs[0].FinishStream()
    model.Wait()
    for r in (rec, recs[0]):
        json.loads(r.Result() or "{}")
    del recs, rec
    model.Wait()
