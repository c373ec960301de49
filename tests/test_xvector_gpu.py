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
