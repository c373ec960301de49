"""Silence weighting of the online i-vector statistics (the reference
Recognizer's UpdateSilenceWeights, src/recognizer.cc:226-237, configured in
src/model.cc:230-231): host restatement (silence.h) against the Python
oracle's restatement, and the weighted-entry machinery of the oracle
extractor.  Parity is unpinned against Kaldi (OnlineSilenceWeighting lives in
the un-vendored Kaldi dependency); these tests pin the two restatements to
each other and to the unweighted path."""
import numpy as np
import pytest

import oracle_py
from conftest import perturbed_stream


def _run_py(calls, sil, sw=1e-3, fss=3):
    s = oracle_py.SilenceWeighting(lambda t: bool(sil[t]), sw, fss)
    out = []
    for ready, first, tids, toks in calls:
        s.compute_current_traceback(tids, toks)
        out.append([(f, float(w)) for f, w in s.get_delta_weights(ready, first)])
    return out


def _random_calls(rng, n_calls=40, ntid=50):
    """A growing best path whose tail (and sometimes older frames) changes
    between calls, as a decoder's traceback does."""
    calls, tids, toks = [], [], []
    ready = 0
    for c in range(n_calls):
        ready += int(rng.integers(0, 25))
        ndec = max(0, (ready - 9) // 3)
        while len(tids) < ndec:
            tids.append(int(rng.integers(1, ntid)))
            toks.append(int(rng.integers(0, 1000)))
        if ndec and rng.random() < 0.5:  # re-route the last k frames
            k = int(rng.integers(1, min(ndec, 150) + 1))
            for i in range(ndec - k, ndec):
                tids[i] = int(rng.integers(1, ntid))
                toks[i] = int(rng.integers(0, 1000))
        calls.append((ready, 0, list(tids[:ndec]), list(toks[:ndec])))
    return calls


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_host_silence_weighting_matches_oracle(seed):
    from vosk import engine
    rng = np.random.default_rng(seed)
    sil = (rng.random(50) < 0.3).astype(np.uint8)
    calls = _random_calls(rng)
    got = engine.silence_weighting_run(calls, sil)
    ref = _run_py(calls, sil)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert [f for f, _ in g] == [f for f, _ in r]
        np.testing.assert_array_equal(np.float32([w for _, w in g]), np.float32([w for _, w in r]))


def test_silence_weighting_semantics():
    sil = np.zeros(10, np.uint8)
    sil[1] = 1
    # no traceback yet: every ready frame gets the silence weight
    out = _run_py([(9, 0, [], [])], sil)[0]
    assert [f for f, _ in out] == list(range(9))
    assert all(w == pytest.approx(1e-3) for _, w in out)
    # traceback: frames 0-1 silence (tid 1), frame 2 speech (tid 2); frames
    # past the traceback repeat the last frame's weight
    out = _run_py([(9, 0, [], []), (15, 0, [1, 1, 2], [5, 6, 7])], sil)[1]
    w = dict(out)
    assert w[6] == pytest.approx(1.0 - 1e-3)  # frame 2: silence -> speech
    assert w[9] == 1.0 and w[12] == 1.0  # new frames repeat frame 2's weight
    assert 0 not in w or w[0] == 0.0
    # an unchanged source token stops the traceback update (Kaldi quirk):
    # frame 2 re-routed with the same source token keeps its old tid
    s = oracle_py.SilenceWeighting(lambda t: bool(sil[t]))
    s.compute_current_traceback([2, 2, 2], [5, 6, 7])
    s.compute_current_traceback([2, 2, 1], [5, 6, 7])
    assert s.info[2][1] == 2
    s.compute_current_traceback([2, 2, 1], [5, 6, 8])
    assert s.info[2][1] == 1
    # the decoder segment's first feature frame offsets the output frames
    out = _run_py([(30, 12, [], [])], sil)[0]
    assert out[0][0] == 12 and out[-1][0] == 12 + 3 * 6 - 1


def test_weighted_entries_with_unit_weights_equal_unweighted(synth_model, test_wave):
    """With silence weight 1 every frame is added once with weight 1 in frame
    order: the weighted path must give the unweighted i-vectors and LLH
    bit for bit (checks the entry/queue machinery end to end)."""
    o = oracle_py.OracleModel(synth_model)
    x = test_wave[:16000 * 3]
    orig = oracle_py.SilenceWeighting.__init__

    def unit(self, f, sw=1e-3, fss=3):
        orig(self, f, 1.0, fss)
    r0 = o.online(x, silence_weighting=False)
    try:
        oracle_py.SilenceWeighting.__init__ = unit
        r1 = o.online(x)
    finally:
        oracle_py.SilenceWeighting.__init__ = orig
    np.testing.assert_array_equal(r1["ivectors"], r0["ivectors"])
    np.testing.assert_array_equal(r1["llh"], r0["llh"])
    # and the real silence weight changes the i-vectors
    r2 = o.online(x)
    assert not np.array_equal(r2["ivectors"], r0["ivectors"])
    assert sum(len(e) for e in r2["entries"]) > 0


def test_silence_weighting_reweights_past_frames(synth_model, test_wave):
    """The full utterance re-weights already accumulated frames, including
    negative deltas: the GPU test over it exercises the history ring, not only
    new frames."""
    o = oracle_py.OracleModel(synth_model)
    ref = o.online(perturbed_stream(test_wave, 1, seconds=10.0), chunk=4000)
    prev, back = -1, 0
    for q, ents in zip(ref["requests"], ref["entries"]):
        back += sum(1 for f, _ in ents if f <= prev)
        prev = max(prev, q)
    assert back > 0
    assert any(w < 0 for ents in ref["entries"] for _, w in ents)
