"""The batch lane's dynamic batching rule (CudaOnlinePipelineDynamicBatcher,
src/batch_model.cc:94-96; BatchModel::LaneLoop): a step waits, bounded, for
the rest of the feeding round by chunk sequence -- every running stream that
pushed chunk n-1 must have pushed chunk n, n being the furthest queued chunk.

The CPU tests drive the rule through the host-only ABI entry; the GPU test
feeds BatchRecognizers the test_gpu_batch.py way with one feeding pause
longer than the bounded wait and checks that only that round is split."""
import time

import numpy as np
import pytest

from conftest import perturbed_stream


def _inc(pushed, taken, ended=None):
    from vosk import engine
    return engine.feeding_round_incomplete(pushed, taken, ended or [0] * len(pushed))


def test_nothing_queued_is_complete():
    assert not _inc([0, 0, 0], [0, 0, 0])
    assert not _inc([4, 4], [4, 4])


def test_waits_for_streams_of_the_round():
    # streams 0, 1 pushed their first chunk; 2, 3 have not yet
    assert _inc([1, 1, 0, 0], [0, 0, 0, 0])
    assert not _inc([1, 1, 1, 1], [0, 0, 0, 0])


def test_split_round_does_not_perpetuate():
    # round 2 split by a pause: streams 0, 1 were stepped, 2, 3 are queued.
    # The second half goes at once (0 and 1 already handed chunk 2) ...
    assert not _inc([2, 2, 2, 2], [2, 2, 1, 1])
    # ... and round 3 waits for every stream again, not for half of them
    assert _inc([3, 3, 2, 2], [2, 2, 2, 2])
    assert not _inc([3, 3, 3, 3], [2, 2, 2, 2])


def test_ended_and_lagging_streams_are_not_waited_for():
    # stream 2 finished its input (FinishStream) at chunk 1
    assert not _inc([2, 2, 1], [1, 1, 1], [0, 0, 1])
    # stream 2 is far behind the round (paused without FinishStream)
    assert not _inc([6, 6, 2], [5, 5, 2])
    # a stream with more than one chunk queued offers its oldest
    assert _inc([3, 2, 1], [1, 1, 1])


N = 24
ROUNDS = 16


@pytest.mark.gpu
def test_feeding_pause_splits_one_round_only(synth_model_noep, test_wave, monkeypatch):
    import vosk
    from vosk import engine
    vosk.SetLogLevel(-1)
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_model_noep)
    model = vosk.BatchModel()
    recs = [vosk.BatchRecognizer(model, 16000) for _ in range(N)]
    data = [np.clip(perturbed_stream(test_wave, 40 + i, seconds=ROUNDS * 0.25 + 1), -32768, 32767)
            .astype("<i2").tobytes() for i in range(N)]
    pause_round = 8  # a round in which every stream pushes a chunk (8160-sample chunks, 4000-sample feeds)
    steps = []
    for r in range(ROUNDS):
        before = engine.batch_batching_counters(model)["steps"]
        for i in range(N):
            recs[i].AcceptWaveform(data[i][r * 8000:(r + 1) * 8000])
            if r == pause_round and i == N // 2:
                time.sleep(0.010)  # longer than the bounded wait's 4 ms without a push
        model.Wait()
        steps.append(engine.batch_batching_counters(model)["steps"] - before)
        for rec in recs:
            while rec.Result():
                pass
    c = engine.batch_batching_counters(model)
    chunk_rounds = [r for r in range(ROUNDS) if ((r + 1) * 4000) // 8160 > (r * 4000) // 8160]
    assert pause_round in chunk_rounds
    # every chunk round but the paused one is one step; the paused one is two
    for r in chunk_rounds:
        assert steps[r] == (2 if r == pause_round else 1), (r, steps)
    assert c["split_rounds"] == 1, c
    for rec in recs:
        rec.FinishStream()
    model.Wait()
    del recs


@pytest.mark.gpu
def test_free_right_after_finish_stream(synth_model_noep, test_wave, monkeypatch):
    """BatchRecognizers freed straight after FinishStream, with no Wait():
    the free waits for the stream's queued chunks and its final result in
    production on the worker pool (BatchModel::Release), so no worker touches
    a freed recognizer.  Repeated over several generations of streams on one
    model, with the model freed before its last recognizers."""
    import gc
    import vosk
    vosk.SetLogLevel(-1)
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_model_noep)
    model = vosk.BatchModel()
    for gen in range(3):
        recs = [vosk.BatchRecognizer(model, 16000) for _ in range(8)]
        for i, rec in enumerate(recs):
            x = perturbed_stream(test_wave, 70 + 8 * gen + i, seconds=2.0 + 0.3 * i)
            rec.AcceptWaveform(np.clip(x, -32768, 32767).astype("<i2").tobytes())
            rec.FinishStream()
        if gen == 2:
            del model  # the recognizers keep the (refcounted) batch model alive
            gc.collect()
        del recs
        gc.collect()


def _decode_batch(vosk, waves, pattern):
    from vosk import engine
    model = vosk.BatchModel()
    recs = [vosk.BatchRecognizer(model, 16000) for _ in waves]
    datas = [np.clip(w, -32768, 32767).astype("<i2").tobytes() for w in waves]
    out = [[] for _ in waves]

    def collect():
        for i, r in enumerate(recs):
            while True:
                res = r.Result()
                if not res:
                    break
                out[i].append(res)

    n = max(len(d) for d in datas)
    for o in range(0, n, 8000):
        for i, r in enumerate(recs):
            if o < len(datas[i]):
                r.AcceptWaveform(datas[i][o:o + 8000])
        if pattern == "wait_per_round":
            model.Wait()
            collect()
    for r in recs:
        r.FinishStream()
    model.Wait()
    collect()
    lanes = [engine.batch_recognizer_lane(r) for r in recs]
    nl = engine.batch_lanes(model)
    counters = engine.batch_batching_counters(model)
    del recs
    del model
    return out, lanes, nl, counters


@pytest.fixture(scope="module")
def lane_streams(synth_model_ep, test_wave):
    import batch_expect
    waves = [perturbed_stream(test_wave, 300 + i, seconds=5.0 + 0.9 * i) for i in range(10)]
    exp = batch_expect.expected(synth_model_ep, waves)
    assert sum(len(r) for r in exp) >= 2 * len(waves)  # the rules fire
    return waves, exp


# (lane devices, feeding pattern, VOSK_AMD_BATCH_SCHEDULE seed; 0 = the
# lane's own schedule)
LANE_CASES = [("0", "wait_per_round", 0), ("0,0", "wait_per_round", 0),
              ("0", "queued_upfront", 0), ("0,0", "queued_upfront", 0),
              ("0", "wait_per_round", 11), ("0,0", "wait_per_round", 12),
              ("0", "queued_upfront", 13), ("0,0", "queued_upfront", 14)]


@pytest.mark.gpu
@pytest.mark.parametrize("devices,pattern,schedule", LANE_CASES,
                         ids=[f"{d.replace(',', '+')}-{p}-s{k}" for d, p, k in LANE_CASES])
def test_lane_configurations_equal_oracle(synth_model_ep, lane_streams, monkeypatch, devices, pattern, schedule):
    """Every stream's result messages -- segment boundaries, words and times
    -- equal the oracle's (tests/batch_expect.py) whatever the lane
    configuration: one lane or two lanes on device 0 (the in-library
    multi-GPU path, admission by PickLane; src/batch_model.cc:23-100), the
    feeding pattern (Wait() per round: in-order steps and split rounds;
    everything queued up front: pipelined steps with resets patched into
    staged jobs), and a seeded random lane schedule (chunks left for later
    steps at random, random in-order / pipelined steps)."""
    import batch_expect
    import vosk
    vosk.SetLogLevel(-1)
    waves, exp = lane_streams
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_model_ep)
    monkeypatch.delenv("VOSK_AMD_DEVICE", raising=False)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    monkeypatch.setenv("VOSK_AMD_BATCH_DEVICES", devices)
    if schedule:
        monkeypatch.setenv("VOSK_AMD_BATCH_SCHEDULE", str(schedule))
    else:
        monkeypatch.delenv("VOSK_AMD_BATCH_SCHEDULE", raising=False)
    out, lanes, nl, counters = _decode_batch(vosk, waves, pattern)
    assert nl == len(devices.split(","))
    assert set(lanes) == set(range(nl)), lanes
    assert counters["merged_probes"] == 0, counters
    for i in range(len(waves)):
        batch_expect.check(out[i], exp[i], f"stream {i} (lane {lanes[i]})")


@pytest.mark.gpu
def test_idle_stream_does_not_stall_the_round(synth_model_noep, test_wave, monkeypatch):
    """A lane waiting for the rest of a feeding round is woken by a push only
    once every stream has a chunk queued (BatchModel::Push); with one
    admitted stream that never feeds, the rounds still complete -- released by
    Wait() and the lane's millisecond polls -- and the fed streams' results
    equal the same streams decoded without the idle one."""
    import vosk
    vosk.SetLogLevel(-1)
    monkeypatch.setenv("VOSK_BATCH_MODEL_DIR", synth_model_noep)
    datas = [np.clip(perturbed_stream(test_wave, 60 + i, seconds=3.0), -32768, 32767).astype("<i2").tobytes()
             for i in range(3)]

    def decode(with_idle):
        model = vosk.BatchModel()
        recs = [vosk.BatchRecognizer(model, 16000) for _ in datas]
        idle = vosk.BatchRecognizer(model, 16000) if with_idle else None
        out = [[] for _ in datas]
        worst = 0.0
        for o in range(0, max(len(d) for d in datas), 8000):
            for r, d in zip(recs, datas):
                if o < len(d):
                    r.AcceptWaveform(d[o:o + 8000])
            t0 = time.perf_counter()
            model.Wait()
            worst = max(worst, time.perf_counter() - t0)
        for r in recs:
            r.FinishStream()
        model.Wait()
        for i, r in enumerate(recs):
            while True:
                res = r.Result()
                if not res:
                    break
                out[i].append(res)
        del recs, idle, model
        return out, worst

    ref, _ = decode(False)
    got, worst = decode(True)
    assert got == ref
    assert worst < 2.0, worst
