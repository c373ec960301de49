"""Online i-vector extraction: the C oracle against the
independent float64 numpy restatement, the chunk schedule, and causality.
Parity unpinned against Kaldi itself (not in the reference); the numpy
restatement follows Kaldi's OnlineIvectorFeature as documented in
vosk-api_amd/tools/np_kaldi.py."""
import os

import numpy as np
import pytest

import np_kaldi as nk
import oracle_py


@pytest.fixture(scope="module")
def oracle(synth_model):
    return oracle_py.OracleModel(synth_model)


def test_ivector_oracle_vs_numpy(oracle, synth_model, test_wave):
    feats = oracle.features(test_wave)
    req = oracle.ivector_requests(feats.shape[0])
    got = oracle.ivector.extract(feats, req)
    ref = nk.IvectorModel(os.path.join(synth_model, "ivector")).extract(feats, req)
    assert got.shape == ref.shape == (len(req), 40)
    # float32 features / LDA / posteriors vs float64 throughout
    assert np.abs(got - ref).max() <= 1e-4 * max(1.0, np.abs(ref).max())
    # the i-vectors move (adaptation is doing something) and stay bounded
    assert np.abs(got[-1] - got[0]).max() > 1e-3
    assert np.isfinite(got).all()


def test_ivector_requests_schedule(oracle):
    fpc, R = oracle.fpc, oracle.right_context
    for T in (1, 50, fpc + R, 829, 3000):
        req = oracle.ivector_requests(T)
        nch = -(-(-(-T // oracle.fss)) // (fpc // oracle.fss))
        assert len(req) == nch
        assert req == sorted(req) and req[-1] == min(nch * fpc + R, T) - 1
        assert all(0 <= f < T for f in req)


def test_ivector_is_causal(oracle, test_wave):
    """An i-vector only depends on frames up to its request + splice context:
    truncating the utterance later leaves it bit-identical."""
    feats = oracle.features(test_wave)
    req = oracle.ivector_requests(feats.shape[0])
    full = oracle.ivector.extract(feats, req)
    T1 = 400
    keep = [f for f in req if f + 3 < T1]
    part = oracle.ivector.extract(feats[:T1], keep)
    np.testing.assert_array_equal(part, full[:len(keep)])


def test_ivector_reaches_llh(oracle, test_wave):
    """The nnet output depends on the chunk's i-vector (the input is wired)."""
    feats = oracle.features(test_wave[:32000])
    a = oracle.loglikes_feats(feats)
    iv = oracle.ivectors(feats)
    ivt, t0 = oracle._ivec_of_time(feats.shape[0], len(iv))
    b = oracle.net.forward(feats, iv + 0.5, ivt, t0)
    assert np.abs(a - b).max() > 1e-3
