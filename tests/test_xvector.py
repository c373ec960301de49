"""Speaker x-vector path on the host (CPU).

The oracle pieces the GPU path is checked against (tests/oracle_xvector.py):
snip-edges=false MFCC framing (reflection at the start, online frame count),
sliding-window CMN against its definition, the x-vector length
normalisation, and the speaker model loading through the C ABI.
"""
import ctypes as C
import os

import numpy as np
import pytest

import oracle_py
import oracle_xvector as OX

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vosk-api_amd", "vosk", "libvosk.so")


def test_snip_edges_false_framing(synth_spk, test_wave):
    o = OX.OracleSpk(synth_spk)
    x = test_wave[:16000]
    f = o.features(x)
    L, S = 400, 160
    # frame t starts at t*S + S/2 - L/2 = t*S - 120, samples before 0 reflected
    pad = x[:120][::-1]
    conf = dict(o.conf)
    conf["snip-edges"] = "true"
    g = oracle_py.mfcc(np.concatenate([pad, x]), conf)
    nf = len(f)
    # online count: frames whose end (t*S - 120 + L) is inside the input
    assert nf == max(t for t in range(200) if t * S - 120 + L <= len(x)) + 1
    np.testing.assert_array_equal(f, g[:nf])


def test_sliding_cmn_definition(synth_spk, test_wave):
    o = OX.OracleSpk(synth_spk)
    f = o.features(test_wave)[:420]
    c = o.cmn(f)
    T = len(f)
    ref = np.zeros(f.shape)
    for t in range(T):
        ws = t - 150
        we = ws + 300
        if ws < 0:
            we -= ws
            ws = 0
        if we > T:
            ws = max(0, ws - (we - T))
            we = T
        ref[t] = f[t] - f[ws:we].astype(np.float64).mean(0)
    np.testing.assert_allclose(c, ref, atol=5e-5)


def test_xvector_oracle_properties(synth_spk, test_wave):
    o = OX.OracleSpk(synth_spk)
    v, n = o.xvector(test_wave, 0, [1] * 10000)
    assert n == len(o.features(test_wave))
    assert v.shape == (64,)
    assert abs(float(np.linalg.norm(v.astype(np.float64))) - 8.0) < 1e-4
    # fewer than 50 selected frames: no vector (src/recognizer.cc:386-389)
    v2, n2 = o.xvector(test_wave, 0, [1] * 16 + [0] * 10000)
    assert v2 is None and n2 == 48
    # a different selection gives a different vector
    v3, _ = o.xvector(test_wave, 30, [1, 0] * 5000)
    assert not np.array_equal(v, v3)


def test_spk_model_loads_through_the_abi(synth_spk, tmp_path):
    lib = C.CDLL(LIB)
    lib.vosk_spk_model_new.restype = C.c_void_p
    lib.vosk_spk_model_new.argtypes = [C.c_char_p]
    lib.vosk_spk_model_free.argtypes = [C.c_void_p]
    lib.vosk_set_log_level(-2)
    h = lib.vosk_spk_model_new(synth_spk.encode())
    assert h
    lib.vosk_spk_model_free(h)
    assert not lib.vosk_spk_model_new(str(tmp_path / "missing").encode())


def test_k_slice_rule():
    """nnet_plan.h GemmKSlices / oracle orc_kslices: K / 256 rounded down to a
    power of two, at most 8 (the streaming kernel's split-K reduction), so
    every K of the recipes (768, 1536, 3000 ...) has a GPU kernel."""
    import ctypes as C
    import oracle_py
    f = oracle_py.lib().orc_kslices
    f.restype = C.c_int
    want = {256: 1, 500: 1, 512: 2, 768: 2, 1024: 4, 1280: 4, 1536: 4, 2048: 8, 3072: 8, 4096: 8, 1000: 1}
    for k, n in want.items():
        assert f(k) == n, k
        assert (k // n) % 32 == 0 or n == 1
