"""Resampling oracle (Kaldi LinearResample restatement, oracle.c) against an
independent float64 numpy restatement, plus signal properties."""
import math

import numpy as np
import pytest

import oracle_py


def np_resample(x, rin, rout, num_zeros=6):
    """float64 restatement of feat/resample.cc (whole signal, flush)."""
    cutoff = 0.5 * min(rin, rout)
    g = math.gcd(rin, rout)
    out_unit, in_unit = rout // g, rin // g
    ww = num_zeros / (2.0 * cutoff)
    tick = rin // g * rout
    interval = len(x) * (tick // rin)
    tpo = tick // rout
    last = interval // tpo
    if last * tpo == interval:
        last -= 1
    nout = last + 1 if interval > 0 else 0
    y = np.zeros(nout)
    for k in range(nout):
        unit, ph = divmod(k, out_unit)
        ot = ph / rout
        lo, hi = math.ceil((ot - ww) * rin), math.floor((ot + ww) * rin)
        j = np.arange(lo, hi + 1)
        dt = j / rin - ot
        win = np.where(np.abs(dt) < ww, 0.5 * (1 + np.cos(2 * np.pi * cutoff / num_zeros * dt)), 0.0)
        with np.errstate(invalid="ignore", divide="ignore"):
            filt = np.where(dt != 0, np.sin(2 * np.pi * cutoff * dt) / (np.pi * dt), 2 * cutoff)
        w = filt * win / rin
        idx = j + unit * in_unit
        ok = (idx >= 0) & (idx < len(x))
        y[k] = np.dot(w[ok], x[idx[ok]])
    return y


@pytest.mark.parametrize("rin", [8000, 22050, 44100, 48000])
def test_resample_vs_numpy(test_wave, rin):
    x = test_wave[:rin // 4].astype(np.float32)  # 0.25 s of signal at rate rin
    got = oracle_py.resample(x, rin, 16000)
    ref = np_resample(x.astype(np.float64), rin, 16000)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 2e-4 * np.abs(ref).max()


def test_resample_lengths():
    lib = oracle_py.lib()
    for rin, n in ((8000, 8000), (44100, 44100), (48000, 1), (22050, 0)):
        assert lib.orc_resample_num_outputs(rin, 16000, n) == (n * 16000 + rin - 1) // rin


def test_resample_preserves_a_tone():
    rin = 44100
    t = np.arange(rin) / rin
    x = (1000 * np.sin(2 * np.pi * 440.0 * t)).astype(np.float32)
    y = oracle_py.resample(x, rin, 16000)
    ty = np.arange(len(y)) / 16000
    mid = slice(200, len(y) - 200)  # away from the edges
    assert np.abs(y[mid] - 1000 * np.sin(2 * np.pi * 440.0 * ty[mid])).max() < 5.0
