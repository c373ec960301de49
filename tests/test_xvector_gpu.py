"""Speaker x-vectors on the GPU vs the CPU oracle.

The GPU path (speaker MFCC, selection + sliding CMN, frame-level TDNN layers
on the GEMM kernels, statistics pooling, head, whitening; xvector.h) is
compared bit-exactly with tests/oracle_xvector.py, directly through
vamd_spk_extract and through the recognizer's result ("spk", "spk_frames",
src/recognizer.cc:470-479) with the selection taken from the oracle's best
path.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from conftest import perturbed_stream
import oracle_py
import oracle_xvector as OX

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vosk_mod():
    import vosk
    vosk.SetLogLevel(-1)
    return vosk


@pytest.fixture(scope="module")
def spk_oracle(synth_spk):
    return OX.OracleSpk(synth_spk)


def _extract(vosk_mod, spk, wave, first, keep, rate=16000):
    so = C.CDLL(os.path.join(os.path.dirname(vosk_mod.__file__), "libvosk.so"))
    so.vamd_spk_extract.restype = C.c_int
    so.vamd_spk_extract.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_void_p,
                                    C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    w = np.ascontiguousarray(wave, np.float32)
    k = np.ascontiguousarray(keep, np.int8)
    out = np.zeros(1024, np.float32)
    nf = C.c_int(0)
    r = so.vamd_spk_extract(spk._handle, w.ctypes.data, len(w), rate, first, k.ctypes.data, len(k),
                            out.ctypes.data, len(out), C.byref(nf))
    assert r >= 0
    return (out[:r].copy() if r > 0 else None), nf.value


@pytest.mark.parametrize("case", ["all", "alternate", "offset", "long", "few"])
def test_xvector_matches_oracle(vosk_mod, synth_spk, spk_oracle, test_wave, case):
    spk = vosk_mod.SpkModel(synth_spk)
    wave, first, keep = test_wave, 0, [1] * 10000
    if case == "alternate":
        keep = [1, 1, 0] * 4000
    elif case == "offset":
        first, keep = 61, [0, 1] * 5000
    elif case == "long":
        wave = perturbed_stream(test_wave, 4, seconds=25.0)
    elif case == "few":
        keep = [1] * 16 + [0] * 10000
    got, n = _extract(vosk_mod, spk, wave, first, keep)
    ref, nr = spk_oracle.xvector(wave, first, keep)
    assert n == nr
    if ref is None:
        assert got is None
        return
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("rate", [8000, 44100])
def test_xvector_other_sample_rates(vosk_mod, synth_spk, spk_oracle, test_wave, rate):
    """Input at another rate goes through the GPU resampler first (Kaldi
    LinearResample, not flushed, as the online speaker front end)."""
    spk = vosk_mod.SpkModel(synth_spk)
    wave = oracle_py.resample(test_wave, 16000, rate)
    got, n = _extract(vosk_mod, spk, wave, 0, [1] * 10000, rate=rate)
    x16 = oracle_py.resample(wave, rate, 16000)[:oracle_py.resample_num_outputs(rate, 16000, len(wave), False)]
    ref, nr = spk_oracle.xvector(x16, 0, [1] * 10000)
    assert n == nr
    np.testing.assert_array_equal(got, ref)


def test_recognizer_result_carries_the_speaker_vector(vosk_mod, synth_model_noep, synth_spk,
                                                      spk_oracle, test_wave):
    """src/recognizer.cc:356-419,470-479: the final result's "spk" is the
    x-vector of the segment's non-silence frames on the final best path."""
    m = vosk_mod.Model(synth_model_noep)
    spk = vosk_mod.SpkModel(synth_spk)
    rec = vosk_mod.KaldiRecognizer(m, 16000, spk)
    data = np.asarray(test_wave, np.float32).astype("<i2").tobytes()
    for i in range(0, len(data), 8000):
        assert rec.AcceptWaveform(data[i:i + 8000]) == 0
    res = json.loads(rec.FinalResult())
    oracle = oracle_py.OracleModel(synth_model_noep)
    path = oracle.online(test_wave, chunk=4000)["decode"]["path"]
    sil = set(int(p) for p in str(oracle.model_conf.get("endpoint.silence-phones", "")).replace(",", ":").split(":") if p)
    g, tm = oracle.graph, oracle.tm
    keep = [0 if int(tm.tid2phone[g.ilabel[a]]) in sil else 1 for a in path if g.ilabel[a] != 0]
    ref, nr = spk_oracle.xvector(test_wave, 0, keep)
    if ref is None:
        assert "spk" not in res
        return
    assert res["spk_frames"] == nr
    np.testing.assert_allclose(np.array(res["spk"], np.float64), ref.astype(np.float64), atol=1e-6)
    # a plain recognizer reports no speaker fields; SetSpkModel adds them
    rec2 = vosk_mod.KaldiRecognizer(m, 16000)
    rec2.SetSpkModel(spk)
    for i in range(0, len(data), 8000):
        rec2.AcceptWaveform(data[i:i + 8000])
    res2 = json.loads(rec2.FinalResult())
    assert res2.get("spk_frames") == nr


def _extract_batch(vosk_mod, spk, reqs, cap=1024):
    """reqs: (wave, rate, first, keep) per utterance -> vamd_spk_extract_batch"""
    so = C.CDLL(os.path.join(os.path.dirname(vosk_mod.__file__), "libvosk.so"))
    so.vamd_spk_extract_batch.restype = C.c_int
    so.vamd_spk_extract_batch.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    n = len(reqs)
    ws = [np.ascontiguousarray(w, np.float32) for w, _, _, _ in reqs]
    ks = [np.ascontiguousarray(k, np.int8) for _, _, _, k in reqs]
    wp = (C.c_void_p * n)(*[w.ctypes.data for w in ws])
    kp = (C.c_void_p * n)(*[k.ctypes.data for k in ks])
    ln = np.array([len(w) for w in ws], np.int64)
    rate = np.array([r for _, r, _, _ in reqs], np.int32)
    first = np.array([f for _, _, f, _ in reqs], np.int32)
    nk = np.array([len(k) for k in ks], np.int32)
    out = np.zeros((n, cap), np.float32)
    nf = np.zeros(n, np.int32)
    st = np.zeros(n, np.int32)
    r = so.vamd_spk_extract_batch(spk._handle, n, wp, ln.ctypes.data, rate.ctypes.data, first.ctypes.data, kp,
                                  nk.ctypes.data, out.ctypes.data, cap, nf.ctypes.data, st.ctypes.data)
    assert r == n
    return [(out[i, :st[i]].copy() if st[i] > 0 else None, int(nf[i])) for i in range(n)]


def _batch_cases(test_wave):
    reqs = []
    for i in range(24):
        secs = [3.0, 6.5, 12.0, 25.0][i % 4] + 0.1 * i
        w = perturbed_stream(test_wave, 900 + i, seconds=secs)
        first = [0, 0, 61, 7][i % 3]
        keep = [[1] * 10000, [1, 1, 0] * 4000, [0, 1] * 5000, [1] * 16 + [0] * 10000][(i // 2) % 4]
        rate = 16000
        if i % 6 == 5:
            rate = [8000, 44100][(i // 6) % 2]
            w = oracle_py.resample(w, 16000, rate)
        reqs.append((w, rate, first, keep))
    return reqs


def test_xvector_batch_matches_oracle_and_single(vosk_mod, synth_spk, spk_oracle, test_wave):
    """24 utterances of 3-27 s (some at 8 / 44.1 kHz, some with too few
    frames) extracted as one batch: each vector equals the oracle's and the
    one vamd_spk_extract gives for the utterance alone, bit for bit."""
    spk = vosk_mod.SpkModel(synth_spk)
    reqs = _batch_cases(test_wave)
    got = _extract_batch(vosk_mod, spk, reqs)
    nvec = 0
    for i, ((w, rate, first, keep), (v, n)) in enumerate(zip(reqs, got)):
        alone, na = _extract(vosk_mod, spk, w, first, keep, rate=rate)
        assert n == na, i
        if rate != 16000:
            w = oracle_py.resample(w, rate, 16000)[:oracle_py.resample_num_outputs(rate, 16000, len(w), False)]
        ref, nr = spk_oracle.xvector(w, first, keep)
        assert n == nr, i
        if ref is None:
            assert v is None and alone is None, i
            continue
        nvec += 1
        np.testing.assert_array_equal(v, ref, err_msg=f"utterance {i}")
        np.testing.assert_array_equal(v, alone, err_msg=f"utterance {i}")
    assert 12 <= nvec < len(reqs)


def test_xvector_batch_split_by_ring_budget(vosk_mod, synth_spk, test_wave, monkeypatch):
    """A ring budget below one long utterance's rings splits the batch into
    several launch sequences; the vectors do not change."""
    reqs = _batch_cases(test_wave)[:8]
    spk = vosk_mod.SpkModel(synth_spk)
    whole = _extract_batch(vosk_mod, spk, reqs)
    monkeypatch.setenv("VOSK_AMD_XVEC_RING_MB", "1")
    spk2 = vosk_mod.SpkModel(synth_spk)
    split = _extract_batch(vosk_mod, spk2, reqs)
    so = C.CDLL(os.path.join(os.path.dirname(vosk_mod.__file__), "libvosk.so"))
    b, u = C.c_longlong(0), C.c_longlong(0)
    assert so.vamd_spk_stats(C.c_void_p(spk2._handle), C.byref(b), C.byref(u), None, None) == 0
    assert u.value == sum(1 for v, _ in whole if v is not None)
    assert b.value > 1
    for (v1, n1), (v2, n2) in zip(whole, split):
        assert n1 == n2
        if v1 is None:
            assert v2 is None
        else:
            np.testing.assert_array_equal(v1, v2)


@pytest.fixture(scope="module")
def sre16_spk(tmp_path_factory):
    """The sre16 x-vector recipe's sizes (tdnn 512 x4 -> 1500, stats pooling,
    embedding 512, 128-dim output): K = 1536 layers split into 4 slices."""
    import make_synth_model as msm
    return msm.make_spk_model(str(tmp_path_factory.mktemp("spk_sre16")), hidden=512, stats_dim=1500,
                              embed=512, out=128)


def test_xvector_recipe_sized_model_matches_oracle(vosk_mod, sre16_spk, test_wave):
    o = OX.OracleSpk(sre16_spk)
    spk = vosk_mod.SpkModel(sre16_spk)
    reqs = [(perturbed_stream(test_wave, 70 + i, seconds=4.0 + 3.0 * i), 16000, 0, [1, 1, 0] * 4000)
            for i in range(3)]
    got = _extract_batch(vosk_mod, spk, reqs)
    for (w, _, first, keep), (v, n) in zip(reqs, got):
        ref, nr = o.xvector(w, first, keep)
        assert n == nr and ref is not None and len(ref) == 128
        np.testing.assert_array_equal(v, ref)
