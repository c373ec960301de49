"""LM rescoring of final results on the host (CPU).

ConstArpa lookups against the n-gram definition, and the C++ rescoring
(csrc/rescore.cc through the host-only lattice pipeline) against its
restatement (tests/oracle_rescore.py) on the oracle decoder's lattices:
subtraction of rescore/G.fst, word determinization, ConstArpa composition,
then the graph scale, MBR and n-best."""
import os

import numpy as np
import pytest

import kaldi_formats as kf
import oracle_lattice as OL
import oracle_py
import oracle_rescore as ORS


def _ngrams(model):
    import make_synth_model as msm
    return msm.add_rescore(model)  # rewrites the same seeded files


def _direct(ng, w, hist, order=3):
    hist = list(hist)[-(order - 1):] if order > 1 else []
    if tuple(hist) + (w,) in ng:
        return np.float32(ng[tuple(hist) + (w,)][0])
    if not hist:
        return np.float32(-np.inf)
    bo = np.float32(ng[tuple(hist)][1]) if tuple(hist) in ng else np.float32(0)
    return np.float32(bo + _direct(ng, w, hist[1:], order))


def test_const_arpa_lookup(synth_model_rescore):
    from vosk import engine
    ng = _ngrams(synth_model_rescore)
    path = os.path.join(synth_model_rescore, "rescore", "G.carpa")
    lm = ORS.ConstArpa(path)
    rng = np.random.default_rng(0)
    words = sorted({w for k in ng for w in k})
    hists = [k for k in ng if len(k) <= 2] + [()]
    for _ in range(400):
        h = list(hists[rng.integers(len(hists))])
        w = int(words[rng.integers(len(words))])
        want = _direct(ng, w, h)
        got_py = lm.logprob(w, h)
        got_c = engine.carpa_logprob(path, w, h)
        # leaves keep their logprob bits minus the lowest one
        assert got_py == pytest.approx(float(want), abs=1e-5)
        assert np.float32(got_c) == got_py


@pytest.mark.parametrize("secs", [2.0, 6.0])
def test_rescoring_matches_restatement(synth_model_rescore, test_wave, secs):
    from vosk import engine
    o = oracle_py.OracleModel(synth_model_rescore)
    wave = test_wave[:int(16000 * secs)]
    r = o.graph.decode(o.loglikes(wave), o.beam, o.max_active, o.min_active, o.beam_delta, True,
                       lattice=True)
    L = OL.raw_from_oracle(r, o.graph, True)
    rd = os.path.join(synth_model_rescore, "rescore")
    engine.set_rescore(os.path.join(rd, "G.fst"), os.path.join(rd, "G.carpa"))
    try:
        got = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, 0.9, 5)
    finally:
        engine.set_rescore(None, None)
    W, Fi = OL.determinize(OL.prune(L, 6.0), o.graph.ilabel, o.graph.olabel)
    G = ORS.prepare_g(kf.read_fst(os.path.join(rd, "G.fst")))
    lm = ORS.ConstArpa(os.path.join(rd, "G.carpa"))
    rr = ORS.rescore(W, Fi, G, lm)
    assert rr is not None and got["rescored"] == 1
    W2, F2 = rr
    assert got["rescored_states"] == len(W2)
    assert got["rescored_arcs"] == sum(len(v) for v in W2)
    W2, F2 = OL.scale_graph(W2, F2, 0.9)
    mb = OL.mbr(W2, F2)
    assert got["mbr"]["words"] == mb["words"]
    np.testing.assert_allclose(got["mbr"]["conf"], mb["conf"], rtol=0, atol=1e-6)
    nb = OL.nbest(W2, F2, 5)
    assert [x["words"] for x in got["nbest"]] == [x["words"] for x in nb]
    np.testing.assert_allclose([x["graph"] + x["acoustic"] for x in got["nbest"]],
                               [x["graph"] + x["acoustic"] for x in nb], rtol=0, atol=1e-3)
    # the rescored best path's graph cost = old graph cost - G.fst + ConstArpa
    # (checked on the first alternative against the unrescored n-best)
    plain = engine.lattice_words(L, o.graph.ilabel, o.graph.olabel, 6.0, 1.0, 50)
    assert got["nbest"][0]["words"] in [x["words"] for x in plain["nbest"]] or len(plain["nbest"]) == 50


def test_const_arpa_kaldi_layout(tmp_path):
    """Hand-built bytes in Kaldi's ConstArpaLm::Write layout (not through
    kaldi_formats.write_const_arpa): the first state at offset 0 and -1 for
    words without a unigram state (<eps> here, as in every real G.carpa)."""
    import struct
    from vosk import engine
    f = lambda x: struct.unpack("<i", struct.pack("<f", x))[0]  # noqa: E731
    leaf = lambda x: f(x) & ~1  # noqa: E731
    lp = {1: -99.0, 2: -1.5, 3: -2.25, 4: -3.5}     # <s> </s> a b
    bo = {1: -0.5, 2: 0.0, 3: -0.75, 4: -1.25}
    lp_ab, lp_sa, bo_sa, lp_sab = -0.625, -1.125, -0.375, -0.3125
    st = [f(lp[1]), f(bo[1]), 1, 3, 2 * (16 - 0) + 1,     # 0: <s> -> (<s> a)
          f(lp[2]), f(bo[2]), 0,                          # 5: </s>
          f(lp[3]), f(bo[3]), 1, 4, leaf(lp_ab),          # 8: a -> leaf (a b)
          f(lp[4]), f(bo[4]), 0,                          # 13: b
          f(lp_sa), f(bo_sa), 1, 4, leaf(lp_sab)]         # 16: <s> a -> leaf (<s> a b)
    uni = [-1, 0, 5, 8, 13]
    b = bytearray(b"\0B")
    tok = lambda t: b.extend(t.encode() + b" ")  # noqa: E731
    i32 = lambda v: b.extend(b"\x04" + struct.pack("<i", v))  # noqa: E731
    i64 = lambda v: b.extend(b"\x08" + struct.pack("<q", v))  # noqa: E731
    tok("<ConstArpaLm>"); tok("<LmInfo>"); i32(1); i32(2); i32(-1); i32(3); tok("</LmInfo>")
    tok("<LmStates>"); i64(len(st)); b.extend(struct.pack(f"<{len(st)}i", *st)); tok("</LmStates>")
    tok("<LmUnigram>"); i32(len(uni))
    for u in uni:
        i64(u)
    tok("</LmUnigram>"); tok("<LmOverflow>"); i32(0); tok("</LmOverflow>"); tok("</ConstArpaLm>")
    path = str(tmp_path / "G.carpa")
    open(path, "wb").write(bytes(b))
    F = np.float32
    unleaf = lambda x: F(struct.unpack("<f", struct.pack("<i", leaf(x)))[0])  # noqa: E731
    want = {(4, (1, 3)): unleaf(lp_sab),             # trigram leaf under the offset-0 root
            (4, (3,)): unleaf(lp_ab),
            (3, (1,)): F(lp_sa),                       # offset-0 state's child
            (3, (4,)): F(bo[4]) + F(lp[3]),            # backoff
            (4, (1,)): F(bo[1]) + F(lp[4]),            # offset-0 state backs off
            (3, (4, 4)): F(bo[4]) + F(lp[3]),          # missing history state
            (2, ()): F(lp[2]), (1, ()): F(lp[1])}
    lm = ORS.ConstArpa(path)
    for (w, h), v in want.items():
        assert lm.logprob(w, list(h)) == v, (w, h)
        assert np.float32(engine.carpa_logprob(path, w, list(h))) == v, (w, h)
