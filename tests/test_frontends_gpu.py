"""GPU parity for the fbank / global-CMVN front ends:
features, i-vectors, LLH and best path bit-identical to the oracle."""
import numpy as np
import pytest

import oracle_py
from conftest import perturbed_stream

pytestmark = pytest.mark.gpu


def _feed(e, s, wave, chunk=3200):
    for i in range(0, len(wave), chunk):
        e.accept(s, wave[i:i + chunk])
        e.advance([s])
    e.accept(s, np.zeros(0, np.float32), finished=True)
    e.advance([s])


@pytest.mark.parametrize("fpc", [21, 51])
def test_frontend_bit_exact(synth_model_frontend, test_wave, fpc):
    from vosk import engine
    o = oracle_py.OracleModel(synth_model_frontend, fpc=fpc)
    e = engine.Engine(synth_model_frontend, frames_per_chunk=fpc, max_streams=4, keep_llh=True)
    s = e.new_stream()
    _feed(e, s, test_wave)
    raw = o.features(test_wave)
    feats = o.nnet_features(raw)
    n = feats.shape[0]
    np.testing.assert_array_equal(e.features(s, n - 64, 64, feats.shape[1]), feats[n - 64:])
    np.testing.assert_array_equal(e.ivectors(s), o.ivectors(raw))
    np.testing.assert_array_equal(e.llh(s), o.loglikes(test_wave))
    arcs, _, _ = e.best_path(s, use_final=True)
    np.testing.assert_array_equal(arcs, o.recognize(test_wave)["path"])


def test_frontend_pipelined_batch(synth_model_frontend, test_wave):
    from vosk import engine
    o = oracle_py.OracleModel(synth_model_frontend, fpc=51)
    n = 4
    e = engine.Engine(synth_model_frontend, frames_per_chunk=51, max_streams=n, keep_llh=True,
                      pipeline=True)
    e.set_step_samples(51 * 160)
    waves = [perturbed_stream(test_wave, i, seconds=2.0 + 0.5 * i) for i in range(n)]
    ss = [e.new_stream() for _ in range(n)]
    for s, w in zip(ss, waves):
        e.preload(s, w, finished=True)
    steps = 0
    while e.step(ss):
        steps += 1
        assert steps < 1000
    for k in range(n):
        np.testing.assert_array_equal(e.llh(ss[k]), o.loglikes(waves[k]), err_msg=f"llh {k}")
