"""Front ends other than plain MFCC (src/model.cc:218-269):
log-fbank features and online CMVN with global stats on the nnet input.
The C oracle against the float64 numpy restatement (parity unpinned vs
Kaldi, which is not in the reference)."""
import numpy as np

import np_kaldi as nk
import oracle_py


def test_fbank_oracle_vs_numpy(test_wave):
    conf = {"num-mel-bins": "40", "low-freq": "20", "high-freq": "-400", "dither": "0"}
    for energy in ("false", "true"):
        c = dict(conf, **{"use-energy": energy})
        got = oracle_py.mfcc(test_wave[:32000], c, fbank=True)
        ref = nk.fbank(test_wave[:32000], nk.MfccOpts(c, fbank=True))
        assert got.shape == ref.shape == (198, 40 + (energy == "true"))
        assert np.abs(got - ref).max() <= 2e-5 * np.abs(ref).max()


def test_online_cmvn_oracle_vs_numpy(test_wave):
    conf = {"num-mel-bins": "40", "num-ceps": "40", "use-energy": "false", "dither": "0"}
    f = oracle_py.mfcc(np.tile(test_wave, 2), conf)  # > 600 frames: the window slides
    g = np.zeros((2, f.shape[1] + 1))
    g[0, :-1] = f[:300].sum(0) * 3.0
    g[0, -1] = 900.0
    got = oracle_py.online_cmvn(f, g)
    ref = nk.online_cmvn(f, g)
    assert f.shape[0] > 1200
    assert np.abs(got - ref).max() <= 2e-5 * np.abs(ref).max()
    # causal: a prefix gives the same rows
    np.testing.assert_array_equal(oracle_py.online_cmvn(f[:700], g), got[:700])


def test_frontend_models_run(synth_model_frontend, test_wave):
    o = oracle_py.OracleModel(synth_model_frontend, fpc=21)
    assert o.global_cmvn is not None
    raw = o.features(test_wave)
    feats = o.nnet_features(raw)
    assert raw.shape == feats.shape == (829, 40)
    assert not np.array_equal(raw, feats)
    r = o.recognize(test_wave)
    assert len(r["words"]) > 0
