"""GPU: silence-weighted online i-vectors (src/recognizer.cc:226-237) against
the oracle's replay of the Recognizer flow.  Per 0.2 s piece the engine
traces back its best path, queues Kaldi-style delta weights, and the next
i-vector requests apply them to the statistics from the per-stream history
ring; i-vectors, log-likelihoods and the best path must match bit for bit."""
import numpy as np
import pytest

import oracle_py

pytestmark = pytest.mark.gpu


def _run_engine(model, wave, chunk, rate=16000):
    from vosk import engine
    e = engine.Engine(model, frames_per_chunk=0, max_streams=2, keep_llh=True)
    s = e.new_stream()
    if rate != 16000:
        e.set_rate(s, rate)
    pos = 0
    for k in oracle_py.recognizer_pieces(len(wave), chunk, rate):
        e.accept(s, wave[pos:pos + k])
        pos += k
        assert e.update_silence_weights(s, 0)
        e.advance([s])
    e.accept(s, np.zeros(0, np.float32), finished=True)
    e.update_silence_weights(s, 0)
    e.advance([s])
    return e, s


@pytest.mark.parametrize("secs,chunk", [(4, 4000), (None, 4000), (None, 16000), ("p1", 4000)])
def test_silence_weighted_stream_matches_oracle(synth_model, test_wave, secs, chunk):
    """("p1": a 10 s perturbed stream whose traceback changes re-weight past
    frames with negative deltas.)"""
    from conftest import perturbed_stream
    x = (test_wave if secs is None else perturbed_stream(test_wave, 1, seconds=10.0) if secs == "p1"
         else test_wave[:16000 * secs])
    o = oracle_py.OracleModel(synth_model)
    ref = o.online(x, chunk=chunk)
    e, s = _run_engine(synth_model, x, chunk)
    iv = e.ivectors(s)
    assert iv.shape == ref["ivectors"].shape, (iv.shape, ref["ivectors"].shape)
    np.testing.assert_array_equal(iv, ref["ivectors"])
    llh = e.llh(s)
    assert llh.shape == ref["llh"].shape
    np.testing.assert_array_equal(llh, ref["llh"])
    arcs, cost, _ = e.best_path(s, use_final=True)
    np.testing.assert_array_equal(arcs, ref["decode"]["path"])

