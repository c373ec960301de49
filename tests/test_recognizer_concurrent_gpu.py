"""Concurrent KaldiRecognizers (one per thread, the reference's usual server
shape: vosk-server runs one recognizer per connection on a thread pool,
src/recognizer.cc:297-323 per call).  Their AcceptWaveform/FinalResult calls
are coalesced into shared batched engine steps (Engine::AdvanceCoalesced);
every stream's results must equal those of the same stream decoded alone.
The second case caps the stream engine at 4 slots so the recognizers spread
over several engines (Model::AllocStreamSlot); the third spreads them over 3
engines from the start (VOSK_AMD_STREAM_ENGINES, the least-loaded engine)."""
import json
import os
import threading

import numpy as np
import pytest

from conftest import perturbed_stream

pytestmark = pytest.mark.gpu


def _pcm(x):
    return np.asarray(x, np.float32).astype("<i2").tobytes()


def _run(rec, data, out, key):
    res = []
    for i in range(0, len(data), 8000):
        if rec.AcceptWaveform(data[i:i + 8000]):
            res.append(json.loads(rec.Result()))
    res.append(json.loads(rec.FinalResult()))
    out[key] = res


@pytest.mark.parametrize("max_streams", [None, 4, "spread3"])
def test_concurrent_recognizers_match_sequential(synth_model_ep, test_wave, max_streams, monkeypatch):
    import vosk
    vosk.SetLogLevel(-1)
    if max_streams == "spread3":
        monkeypatch.setenv("VOSK_AMD_STREAM_ENGINES", "3")
        monkeypatch.setenv("VOSK_AMD_MAX_STREAMS", "8")
    elif max_streams:
        monkeypatch.setenv("VOSK_AMD_MAX_STREAMS", str(max_streams))
    waves = [_pcm(perturbed_stream(test_wave, 40 + i, seconds=8.0)) for i in range(10)]
    m = vosk.Model(synth_model_ep)

    alone = {}
    for i, d in enumerate(waves):
        rec = vosk.KaldiRecognizer(m, 16000)
        rec.SetWords(True)
        _run(rec, d, alone, i)
        del rec

    recs = []
    for _ in waves:
        r = vosk.KaldiRecognizer(m, 16000)
        r.SetWords(True)
        recs.append(r)
    together, errs = {}, []

    def work(i):
        try:
            _run(recs[i], waves[i], together, i)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(waves))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th)
    assert not errs, errs
    for i in range(len(waves)):
        assert len(together[i]) == len(alone[i]) >= 2
        for a, b in zip(alone[i], together[i]):
            assert a["text"] == b["text"]
            wa, wb = a.get("result", []), b.get("result", [])
            assert [w["word"] for w in wa] == [w["word"] for w in wb]
            for x, y in zip(wa, wb):
                assert x["start"] == y["start"] and x["end"] == y["end"]
                assert x["conf"] == pytest.approx(y["conf"], abs=1e-5)


def _script(seed, nbytes):
    """A seeded caller: AcceptWaveform calls of 0.0625-0.75 s (one to four
    0.2-s pieces, so batched passes carry requests over), PartialResult after
    some, one Reset for some streams, Result on endpoints, FinalResult."""
    rng = np.random.default_rng(seed)
    ops, o = [], 0
    reset_at = int(rng.integers(nbytes // 3, 2 * nbytes // 3)) if seed % 3 == 0 else -1
    while o < nbytes:
        n = int(rng.choice([2000, 4000, 8000, 12000, 24000]))
        ops.append(("accept", o, min(o + n, nbytes)))
        if rng.random() < 0.35:
            ops.append(("partial",))
        if reset_at >= 0 and o <= reset_at < o + n:
            ops.append(("reset",))
        o += n
    ops.append(("final",))
    return ops


def _play(rec, data, ops):
    out = []
    for op in ops:
        if op[0] == "accept":
            if rec.AcceptWaveform(data[op[1]:op[2]]):
                out.append(("result", json.loads(rec.Result())))
        elif op[0] == "partial":
            out.append(("partial", json.loads(rec.PartialResult())))
        elif op[0] == "reset":
            rec.Reset()
        else:
            out.append(("final", json.loads(rec.FinalResult())))
    return out


def test_concurrent_mixed_calls_match_sequential(synth_model_ep, test_wave):
    """Twelve recognizers on twelve threads with their own call sizes,
    partial results (partial words on for half of them), resets and endpoint
    results: every output -- partials included, word times and confidences --
    equals the same calls made alone (the batched passes' carried requests
    and the background lattice replays change nothing)."""
    import vosk
    vosk.SetLogLevel(-1)
    n = 12
    waves = [_pcm(perturbed_stream(test_wave, 70 + i, seconds=6.0)) for i in range(n)]
    scripts = [_script(100 + i, len(waves[i])) for i in range(n)]
    m = vosk.Model(synth_model_ep)

    def make(i):
        r = vosk.KaldiRecognizer(m, 16000)
        r.SetWords(True)
        r.SetPartialWords(i % 2 == 0)
        return r

    alone = []
    for i in range(n):
        r = make(i)
        alone.append(_play(r, waves[i], scripts[i]))
        del r
    recs = [make(i) for i in range(n)]
    together, errs = [None] * n, []

    def work(i):
        try:
            together[i] = _play(recs[i], waves[i], scripts[i])
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    assert not any(t.is_alive() for t in th)
    assert not errs, errs
    for i in range(n):
        assert [k for k, _ in together[i]] == [k for k, _ in alone[i]], i
        assert together[i] == alone[i], i
    assert sum(1 for i in range(n) for k, v in alone[i] if k == "partial" and v.get("partial")) > n
